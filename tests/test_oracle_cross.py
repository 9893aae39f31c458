"""The two independent oracle restatements must agree.

naive  : exact-integer loops over NCHW/OIHW straight from the op definitions.
mnn    : the reference's own data flow -- C4 layout, per-call weight reorder, 4-pixel
         im2col tiles, 16x4 GEMM unit, and the grad graph (x^T / dy^T, LeftPoolGrad
         dilation, extra pad, rot180 of w^T) of grad/NITI_Conv_Int8_Grad.cpp.
"""
import numpy as np
import pytest

# (n, c_in, h, w, c_out, k, stride, pad)
GEOMS = [
    (4, 1, 28, 28, 20, 5, 1, 0),     # LeNet conv1 (batch cut)
    (4, 20, 12, 12, 52, 5, 1, 0),    # LeNet conv2
    (4, 832, 1, 1, 500, 1, 1, 0),    # LeNet ip1 (1x1)
    (4, 500, 1, 1, 12, 1, 1, 0),     # LeNet ip2
    (3, 3, 16, 16, 64, 3, 1, 1),     # VGG L1 shape, cut
    (2, 64, 8, 8, 128, 3, 1, 1),     # VGG L2 shape, cut
    (5, 6, 9, 9, 8, 3, 2, 1),        # stride 2, odd sizes
    (2, 4, 8, 8, 4, 3, 2, 1),        # stride 2, even
    (7, 5, 6, 7, 12, 3, 1, 1),       # ragged batch / channels
]


@pytest.mark.parametrize("geo", GEOMS)
def test_fwd_naive_vs_mnn(oracle, geo):
    n, ci, h, w, co, k, s, p = geo
    rng = np.random.default_rng(17)
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    x = oracle.synth_x(rng, (n, ci, h, w))
    wt, wscale = oracle.synth_w(rng, (co, ci, k, k))
    y0, e0, acc, st = oracle.conv_fwd(g, x, wt, -7, wscale)
    y1, e1, _ = oracle.mnn_conv_fwd(g, x, wt, -7, wscale)
    assert st.overflow == 0
    assert e0 == e1
    assert np.array_equal(y0, y1)
    if st.guard == 0:  # float32 accumulation is exact below 2^24
        y2, e2, _ = oracle.mnn_conv_fwd(g, x, wt, -7, wscale, acc_mode=oracle.ACC_F32_SEQ, threads=3)
        assert e2 == e0 and np.array_equal(y2, y0)


@pytest.mark.parametrize("geo", GEOMS)
def test_wgrad_naive_vs_mnn(oracle, geo):
    n, ci, h, w, co, k, s, p = geo
    rng = np.random.default_rng(18)
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    x = oracle.synth_x(rng, (n, ci, h, w))
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    dw0, bw0, acc0, st = oracle.conv_wgrad(g, x, dy)
    dw1, bw1, acc1 = oracle.mnn_conv_wgrad(g, x, dy)
    assert np.array_equal(acc0, acc1)
    assert bw0 == bw1 and np.array_equal(dw0, dw1)
    assert np.abs(dw0.astype(int)).max() <= 4


@pytest.mark.parametrize("geo", [g for g in GEOMS if g[2] > 1])
def test_dgrad_naive_vs_mnn(oracle, geo):
    n, ci, h, w, co, k, s, p = geo
    rng = np.random.default_rng(19)
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    if s == 2 and (w - ((w + 2 * p - k + 1) + 2 * p - k + 1)) % 2:
        pytest.skip("reference extra-pad arithmetic undefined for this shape")
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    wt, _ = oracle.synth_w(rng, (co, ci, k, k))
    dx0, inc0, acc0, st = oracle.conv_dgrad(g, dy, wt)
    dx1, inc1, acc1 = oracle.mnn_conv_dgrad(g, dy, wt)
    assert np.array_equal(acc0, acc1)
    assert inc0 == inc1 and np.array_equal(dx0, dx1)


def test_matmul_equals_wgrad_gemm(oracle):
    """NITI_Matmul_Int8 on the backprop-filter geometry == the weight-gradient GEMM
    (NITI_GeometryConv2DBackPropFilter_Int8.cpp:40-121), with its own bw-3 rule."""
    rng = np.random.default_rng(20)
    n, ci, h, w, co, k, p = 3, 5, 6, 6, 8, 3, 1
    g = oracle.geom(n, ci, h, w, co, k, pad=p)
    x = oracle.synth_x(rng, (n, ci, h, w))
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    # B = im2col(x): [ci*kh*kw][n*oh*ow];  A = dy as [co][n*oh*ow]
    xp = np.pad(x, ((0, 0), (0, 0), (p, p), (p, p)))
    B = np.zeros((ci, k, k, n, g.oh, g.ow), np.int8)
    for ky in range(k):
        for kx in range(k):
            B[:, ky, kx] = xp[:, :, ky:ky + g.oh, kx:kx + g.ow].transpose(1, 0, 2, 3)
    B = B.reshape(ci * k * k, -1)
    A = dy.transpose(1, 0, 2, 3).reshape(co, -1)
    dwm, bwm, accm, _ = oracle.matmul(B, A)
    accw, _ = oracle.conv_wgrad_acc(g, x, dy)
    assert np.array_equal(accm.T.reshape(co, ci, k, k), accw)
    q, bw = oracle.requant_matmul(accw)
    assert bw == bwm and np.array_equal(dwm.reshape(co, ci, k, k), q)


def test_guard_and_float_divergence(oracle):
    """Stress inputs push sum|x*w| past 2^24: the guard fires, and that is exactly where the
    reference's float32 accumulation may differ from the exact sum."""
    rng = np.random.default_rng(21)
    g = oracle.geom(2, 1024, 6, 6, 8, 3, pad=1)
    x = oracle.synth_stress(rng, (2, 1024, 6, 6))
    w = oracle.synth_stress(rng, (8, 1024, 3, 3))
    acc, st = oracle.conv_fwd_acc(g, x, w)
    assert st.guard > 0 and st.overflow == 0


def test_threads_do_not_change_results(oracle):
    rng = np.random.default_rng(22)
    g = oracle.geom(6, 8, 10, 10, 16, 3, pad=1)
    x = oracle.synth_x(rng, (6, 8, 10, 10))
    w, ws = oracle.synth_w(rng, (16, 8, 3, 3))
    a = oracle.mnn_conv_fwd(g, x, w, -7, ws, threads=1)
    b = oracle.mnn_conv_fwd(g, x, w, -7, ws, threads=4)
    assert np.array_equal(a[0], b[0]) and a[1] == b[1]
