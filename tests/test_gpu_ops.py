"""GPU parity: every HIP kernel / C-ABI entry point against the CPU oracle, bit for bit.

All calls go through libniti_hip.so (include/niti_hip.h).  The oracle is the checker only.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GEOMS = [
    (4, 1, 28, 28, 20, 5, 1, 0),     # LeNet conv1 (batch cut)
    (4, 20, 12, 12, 52, 5, 1, 0),    # LeNet conv2
    (4, 832, 1, 1, 500, 1, 1, 0),    # LeNet ip1
    (4, 500, 1, 1, 12, 1, 1, 0),     # LeNet ip2
    (3, 3, 16, 16, 64, 3, 1, 1),     # VGG L1 shape
    (2, 64, 8, 8, 128, 3, 1, 1),     # VGG L2 shape
    (17, 256, 4, 4, 256, 3, 1, 1),   # VGG mid, ragged batch
    (5, 6, 9, 9, 8, 3, 2, 1),        # stride 2
    (7, 5, 6, 7, 12, 3, 1, 1),       # ragged everything
    (3, 40, 7, 5, 36, 3, 1, 0),      # non-square, no pad
    (3, 8, 9, 9, 12, 3, 2, 1),       # stride 2, channels % 4 == 0
    # the conv / deconv Executions take the fused row kernel where the geometry allows (stride-1
    # pad-1 3x3, square 2/4/8/16 maps, c_out padded to a multiple of 32): ragged channels, and the
    # K-split 2x2 form (128 input channels)
    (5, 40, 8, 8, 52, 3, 1, 1),
    (9, 96, 2, 2, 128, 3, 1, 1),
    (9, 128, 2, 2, 92, 3, 1, 1),
]


@pytest.fixture(scope="module")
def T():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import niti_amd  # noqa: F401  (fails loudly without the HIP library)
    return torch


@pytest.fixture(scope="module")
def ops(T):
    from niti_amd import ops
    return ops


def dev(T, a, dtype=None):
    return T.from_numpy(np.ascontiguousarray(a)).to("cuda")


def zeros_u32(T):
    return T.zeros(2048, dtype=T.int32, device="cuda")  # NITI_MAX_WORDS words per range


def i8s(T, v):
    return T.tensor([v], dtype=T.int8, device="cuda")


# --------------------------------------------------------------------------- GEMM core
@pytest.mark.parametrize("m,o,k", [(1, 1, 1), (37, 29, 100), (128, 128, 64), (300, 200, 777), (5, 700, 4100),
                                   (64, 144, 65536), (256, 2304, 16384)])
@pytest.mark.parametrize("split", [False, True])
def test_matmul_acc_exact(T, ops, m, o, k, split):
    rng = np.random.default_rng(m * 7 + o + k)
    B = rng.integers(-128, 128, (m, k), dtype=np.int16).astype(np.int8)
    A = rng.integers(-128, 128, (o, k), dtype=np.int16).astype(np.int8)
    k16 = (k + 15) // 16 * 16
    Bp = np.zeros((m, k16), np.int8)
    Bp[:, :k] = B
    Ap = np.zeros((o, k16), np.int8)
    Ap[:, :k] = A
    ldc = (o + 15) // 16 * 16
    amax = zeros_u32(T)
    acc = ops.matmul_acc(dev(T, Bp), dev(T, Ap), ldc, amax=amax, use_workspace=split)
    want = B.astype(np.int64) @ A.astype(np.int64).T
    got = acc.cpu().numpy()
    assert np.array_equal(got[:, :o], want)
    assert not got[:, o:].any()
    assert ops.range_max(amax) == int(np.abs(want).max())


# --------------------------------------------------------------------------- native conv ops
def nchw_to_nhwc_acc(a):
    return np.ascontiguousarray(a.transpose(0, 2, 3, 1)).reshape(-1, a.shape[1])


@pytest.mark.parametrize("geo", GEOMS)
def test_conv_fwd_native(T, ops, oracle, geo):
    n, ci, h, w, co, k, s, p = geo
    rng = np.random.default_rng(101)
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    x = oracle.synth_x(rng, (n, ci, h, w))
    wt, ws = oracle.synth_w(rng, (co, ci, k, k))
    y_ref, e_ref, acc_ref, _ = oracle.conv_fwd(g, x, wt, -7, ws)
    gg = ops.geom(n, ci, h, w, co, k, stride=s, pad=p)
    x16 = ops.nchw_to_nhwc16(dev(T, x))
    w16 = ops.oihw_to_ohwi16(dev(T, wt))
    amax = zeros_u32(T)
    acc = ops.conv_fwd_acc(gg, x16, w16, amax)
    got = acc.cpu().numpy()
    assert np.array_equal(got[:, :co], nchw_to_nhwc_acc(acc_ref))
    assert not got[:, co:].any()
    assert ops.range_max(amax) == int(np.abs(acc_ref.astype(np.int64)).max())
    e_out = i8s(T, 0)
    y16 = ops.requant_act(acc, amax, exp_in=i8s(T, -7), wscale=i8s(T, ws), exp_out=e_out)
    y = y16.cpu().numpy()[:, :co].reshape(n, g.oh, g.ow, co).transpose(0, 3, 1, 2)
    assert np.array_equal(y, y_ref)
    assert int(e_out.item()) == e_ref


@pytest.mark.parametrize("geo", GEOMS)
def test_conv_dgrad_native(T, ops, oracle, geo):
    n, ci, h, w, co, k, s, p = geo
    rng = np.random.default_rng(102)
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    wt, _ = oracle.synth_w(rng, (co, ci, k, k))
    dx_ref, inc_ref, acc_ref, _ = oracle.conv_dgrad(g, dy, wt)
    gg = ops.geom(n, ci, h, w, co, k, stride=s, pad=p)
    dy16 = ops.nchw_to_nhwc16(dev(T, dy))
    w16 = ops.oihw_to_ohwi16(dev(T, wt))
    wT = ops.ohwi16_to_ihwo16(w16, ci)
    amax = zeros_u32(T)
    acc = ops.conv_dgrad_acc(gg, dy16, wT, amax)
    got = acc.cpu().numpy()
    assert np.array_equal(got[:, :ci], nchw_to_nhwc_acc(acc_ref))
    dx16 = ops.requant_act(acc, amax)
    dx = dx16.cpu().numpy()[:, :ci].reshape(n, h, w, ci).transpose(0, 3, 1, 2)
    assert np.array_equal(dx, dx_ref)


@pytest.mark.parametrize("geo", GEOMS)
def test_conv_wgrad_native(T, ops, oracle, geo):
    n, ci, h, w, co, k, s, p = geo
    rng = np.random.default_rng(103)
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    x = oracle.synth_x(rng, (n, ci, h, w))
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    dw_ref, bw_ref, acc_ref, _ = oracle.conv_wgrad(g, x, dy)
    gg = ops.geom(n, ci, h, w, co, k, stride=s, pad=p)
    xT = ops.nchw_to_nhwc16(dev(T, x))
    dyT = ops.nchw_to_nhwc16(dev(T, dy))
    acc = ops.conv_wgrad_acc(gg, xT, dyT)
    got = acc.cpu().numpy()  # [co][kh][kw][cip]
    assert np.array_equal(got[..., :ci].transpose(0, 3, 1, 2), acc_ref)
    assert not got[..., ci:].any()
    amax = zeros_u32(T)
    ops.absmax(acc, amax)
    w16 = T.zeros(acc.shape, dtype=T.int8, device="cuda")
    gq = ops.requant_grad(acc, amax, rule=2, w_update=w16)
    assert np.array_equal(gq.cpu().numpy()[..., :ci].transpose(0, 3, 1, 2), dw_ref)
    # fused SGD: 0 - g, clipped
    assert np.array_equal(w16.cpu().numpy()[..., :ci].transpose(0, 3, 1, 2),
                          oracle.sgd_update(np.zeros_like(dw_ref), dw_ref))
    # tiled SGD kernel: w <- clip(w - g) in OHWI16 plus the transposed IHWO16 copy
    rng2 = np.random.default_rng(104)
    w0, _ = oracle.synth_w(rng2, (co, ci, k, k))
    w16b = ops.oihw_to_ohwi16(dev(T, w0))
    wT, g2 = ops.sgd_update(acc, amax, w16b, ci, rule=2)
    w_new = oracle.sgd_update(w0, dw_ref)
    assert np.array_equal(g2.cpu().numpy()[..., :ci].transpose(0, 3, 1, 2), dw_ref)
    assert np.array_equal(w16b.cpu().numpy()[..., :ci].transpose(0, 3, 1, 2), w_new)
    assert not w16b.cpu().numpy()[..., ci:].any()
    wTn = wT.cpu().numpy()  # [ci][kh][kw][cop]
    assert np.array_equal(wTn[..., :co].transpose(3, 0, 1, 2), w_new)
    assert not wTn[..., co:].any()


# tap-sharing weight gradient (wgrad_taps_kernel): every step mode and split plan
TAPS_GEOMS = [
    (3, 64, 8, 8, 128, 1),     # band: one 8x8 image per 64-pixel step
    (1, 32, 16, 16, 64, 1),    # band: 4 rows of a 16x16 image
    (1, 32, 32, 32, 64, 1),    # band: 2 rows of a 32x32 image (two-KiB region DMA per wave)
    (8, 64, 4, 4, 64, 1),      # whole images: 4 per step
    (16, 32, 2, 2, 128, 1),    # whole images: 16 per step
    (2, 32, 10, 10, 50, 0),    # no padding (10x10 -> 8x8), c_out not a multiple of 64
    (4, 96, 8, 8, 64, 1),      # 3 input-channel tiles
    # segment / 4-row tile modes (rows that are not whole 64-pixel steps; tiles where H % 4 == 0):
    # 16-pixel segments ...
    (2, 32, 48, 48, 64, 1),    # 3 per row
    (1, 32, 112, 112, 64, 1),  # 7 per row (VGG-16 conv2 maps)
    # ... and 14-pixel segments (two zero slots of 16)
    (3, 32, 28, 28, 64, 1),    # 2 per row
    (1, 64, 56, 56, 64, 1),    # 4 per row (VGG-16 conv3 / ResNet-18 layer1 maps)
    (5, 64, 14, 14, 128, 1),   # 1 per row, 70 segments: a partial last step
    (2, 32, 28, 28, 50, 1),    # c_out not a multiple of 64
    (1, 128, 56, 56, 64, 1),   # 4-row tiles at 128 input channels (four ci tiles)
]


@pytest.mark.parametrize("geo", TAPS_GEOMS)
@pytest.mark.parametrize("splits", ["", "1", "3"])
def test_conv_wgrad_taps(T, ops, oracle, geo, splits, monkeypatch):
    n, ci, h, w, co, p = geo
    rng = np.random.default_rng(211)
    g = oracle.geom(n, ci, h, w, co, 3, stride=1, pad=p)
    x = rng.integers(-127, 128, (n, ci, h, w)).astype(np.int8)
    dy = rng.integers(-127, 128, (n, co, g.oh, g.ow)).astype(np.int8)
    _, _, acc_ref, _ = oracle.conv_wgrad(g, x, dy)
    gg = ops.geom(n, ci, h, w, co, 3, stride=1, pad=p)
    assert ops.wgrad_taps_ok(gg)
    xT = ops.nchw_to_nhwc16(dev(T, x))
    dyT = ops.nchw_to_nhwc16(dev(T, dy))
    if splits:
        monkeypatch.setenv("NITI_DIAG_SPLITS", splits)
    amax = zeros_u32(T)
    acc = ops.conv_wgrad_acc(gg, xT, dyT, amax)
    got = acc.cpu().numpy()
    assert np.array_equal(got[..., :ci].transpose(0, 3, 1, 2), acc_ref)
    assert not got[..., ci:].any()
    assert ops.range_max(amax) == int(np.abs(acc_ref.astype(np.int64)).max())
    monkeypatch.setenv("NITI_DIAG_NO_TAPS", "1")  # the generic K-major GEMM agrees bit for bit
    assert np.array_equal(ops.conv_wgrad_acc(gg, xT, dyT).cpu().numpy(), got)


# --------------------------------------------------------------------------- drop-in Executions
def _c4_dims(a):
    return list(a.shape)


@pytest.mark.parametrize("geo", [gg for gg in GEOMS if gg[4] % 4 == 0])
def test_exec_conv_int8(T, ops, oracle, geo):
    import niti_amd
    n, ci, h, w, co, k, s, p = geo
    rng = np.random.default_rng(201)
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    x = oracle.synth_x(rng, (n, ci, h, w))
    wt, ws = oracle.synth_w(rng, (co, ci, k, k))
    y_ref, e_ref, y4_ref = oracle.mnn_conv_fwd(g, x, wt, -7, ws)
    x4 = dev(T, oracle.nchw_to_c4(x))
    y4 = T.zeros(y4_ref.shape, dtype=T.int8, device="cuda")
    e_in, wsc, e_out = i8s(T, -7), i8s(T, ws), i8s(T, 0)
    wd = dev(T, wt)
    ex = ops.NITIExecution(niti_amd.OP_CONV_INT8, ops.conv_common(k, stride=s, pad=p, input_count=ci, output_count=co))
    ins = [ops.tensor(x4, (n, ci, h, w), niti_amd.FORMAT_NC4HW4), ops.tensor(wd, (co, ci, k, k)),
           ops.tensor(e_in, (1, 1, 1, 1)), ops.tensor(wsc, (1, 1, 1, 1))]
    outs = [ops.tensor(y4, (n, co, g.oh, g.ow), niti_amd.FORMAT_NC4HW4), ops.tensor(e_out, (1, 1, 1, 1))]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    assert np.array_equal(y4.cpu().numpy(), y4_ref)
    assert int(e_out.item()) == e_ref


def test_exec_conv_int8_rejects_unaligned_channels(T, ops):
    import niti_amd
    x4 = T.zeros((1, 1, 5, 5, 4), dtype=T.int8, device="cuda")
    w = T.zeros((6, 3, 3, 3), dtype=T.int8, device="cuda")
    y4 = T.zeros((2, 1, 3, 3, 4), dtype=T.int8, device="cuda")
    e = i8s(T, 0)
    ex = ops.NITIExecution(niti_amd.OP_CONV_INT8, ops.conv_common(3))
    ins = [ops.tensor(x4, (1, 3, 5, 5), 2), ops.tensor(w, (6, 3, 3, 3)), ops.tensor(e, (1,)), ops.tensor(e, (1,))]
    outs = [ops.tensor(y4, (1, 6, 3, 3), 2), ops.tensor(e, (1,))]
    assert ex.resize(ins, outs) == 2  # NOT_SUPPORT: C_out % 4 != 0 (reference acc overflow)


@pytest.mark.parametrize("geo", [gg for gg in GEOMS if gg[2] > 1 and gg[1] % 4 == 0])
def test_exec_deconv_int8(T, ops, oracle, geo):
    """NITI_DeConv_Int8 on the tensors the grad graph hands it: pad(dilate(dy)) and w^T."""
    import niti_amd
    n, ci, h, w, co, k, s, p = geo
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    if s == 2 and (w - ((w + 2 * p - k + 1) + 2 * p - k + 1)) % 2:
        pytest.skip("reference extra-pad arithmetic undefined for this shape")
    rng = np.random.default_rng(202)
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    wt, _ = oracle.synth_w(rng, (co, ci, k, k))
    dx_ref, _, _ = oracle.mnn_conv_dgrad(g, dy, wt)
    # build the graph-side inputs exactly as grad/NITI_Conv_Int8_Grad.cpp:86-120 does
    d = dy
    if s == 2:
        ow1 = w + 2 * p - k + 1
        dd = np.zeros((n, co, ow1, ow1), np.int8)
        dd[:, :, ::2, ::2][:, :, :g.oh, :g.ow] = dy
        d = dd
    e = (w - (d.shape[3] + 2 * p - k + 1)) // 2
    if e:
        d = np.pad(d, ((0, 0), (0, 0), (e, e), (e, e)))
    wT = np.ascontiguousarray(wt.transpose(1, 0, 2, 3))
    d4 = dev(T, oracle.nchw_to_c4(d))
    out4 = T.zeros(((ci + 3) // 4, n, h, w, 4), dtype=T.int8, device="cuda")
    ex = ops.NITIExecution(niti_amd.OP_DECONV_INT8, ops.conv_common(k, stride=1, pad=p, input_count=co,
                                                                     output_count=ci))
    ins = [ops.tensor(d4, (n, co, d.shape[2], d.shape[3]), 2), ops.tensor(dev(T, wT), (ci, co, k, k))]
    outs = [ops.tensor(out4, (n, ci, h, w), 2)]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    assert np.array_equal(oracle.c4_to_nchw(out4.cpu().numpy(), ci), dx_ref)


@pytest.mark.parametrize("geo", [gg for gg in GEOMS if gg[4] % 4 == 0])
def test_exec_gradient_conv_int8(T, ops, oracle, geo):
    import niti_amd
    n, ci, h, w, co, k, s, p = geo
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    rng = np.random.default_rng(203)
    x = oracle.synth_x(rng, (n, ci, h, w))
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    dw_ref, bw_ref, _ = oracle.mnn_conv_wgrad(g, x, dy)
    d = dy
    if s == 2:
        ow1 = w + 2 * p - k + 1
        dd = np.zeros((n, co, ow1, ow1), np.int8)
        dd[:, :, ::2, ::2][:, :, :g.oh, :g.ow] = dy
        d = dd
    xT4 = oracle.nchw_to_c4(np.ascontiguousarray(x.transpose(1, 0, 2, 3)))   # C4(x^T)
    dyT = np.ascontiguousarray(d.transpose(1, 0, 2, 3))                       # dy^T NCHW
    out4 = T.zeros(((co + 3) // 4, ci, k, k, 4), dtype=T.int8, device="cuda")
    ex = ops.NITIExecution(niti_amd.OP_GRADIENT_CONV_INT8,
                           ops.conv_common((d.shape[3], d.shape[2]), stride=1, pad=p, input_count=n, output_count=co))
    ins = [ops.tensor(dev(T, xT4), (ci, n, h, w), 2), ops.tensor(dev(T, dyT), (co, n, d.shape[2], d.shape[3]))]
    outs = [ops.tensor(out4, (ci, co, k, k), 2)]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    got = oracle.c4_to_nchw(out4.cpu().numpy(), co)  # [ci][co][k][k]
    assert np.array_equal(got.transpose(1, 0, 2, 3), dw_ref)


@pytest.mark.parametrize("m,o,k", [(27, 64, 3 * 256), (500, 12, 64), (4608, 32, 70)])
def test_exec_matmul_int8(T, ops, oracle, m, o, k):
    import niti_amd
    rng = np.random.default_rng(204)
    B = oracle.synth_x(rng, (m, k))
    A = oracle.synth_dy(rng, (o, k))
    dwT_ref, bw, acc, _ = oracle.matmul(B, A)  # dwT_ref [o][m]
    out = T.zeros((m, o), dtype=T.int8, device="cuda")
    ex = ops.NITIExecution(niti_amd.OP_MATMUL_INT8, None)
    ins = [ops.tensor(dev(T, B), (m, k)), ops.tensor(dev(T, A), (o, k))]
    outs = [ops.tensor(out, (m, o))]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    assert np.array_equal(out.cpu().numpy().T, dwT_ref)


@pytest.mark.parametrize("op", [818, 810, 819, 820])
@pytest.mark.parametrize("geo", [GEOMS[1], GEOMS[4], GEOMS[7]])
def test_exec_dsp_matmul_gradient(T, ops, oracle, geo, op):
    """818, and 810 / 819 / 820 (GRADIENTCONV, MATMUL, PARALLEL_GRADIENTCONV: their common carries dy's OH x OW
    as the kernel; ShapeNITI_Conv_Int8.cpp:146-233 sizes all three)."""
    import niti_amd
    n, ci, h, w, co, k, s, p = geo
    if op != 818 and s != 1:
        pytest.skip("the graph emits 820 only for stride 1")
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    rng = np.random.default_rng(205)
    x = oracle.synth_x(rng, (n, ci, h, w))
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    dw_ref, _, _, _ = oracle.conv_wgrad(g, x, dy)
    out = T.zeros((k, k, ci, co), dtype=T.int8, device="cuda")
    ex = ops.NITIExecution(op, ops.conv_common(k if op == 818 else (g.oh, g.ow), stride=s, pad=p))
    ins = [ops.tensor(dev(T, x.transpose(0, 2, 3, 1)), (n, ci, h, w), niti_amd.FORMAT_NHWC),
           ops.tensor(dev(T, dy.transpose(0, 2, 3, 1)), (n, co, g.oh, g.ow), niti_amd.FORMAT_NHWC)]
    outs = [ops.tensor(out, (k, k, ci, co))]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    assert np.array_equal(out.cpu().numpy().transpose(3, 2, 0, 1), dw_ref)


@pytest.mark.parametrize("geo", GEOMS)
def test_exec_dsp_conv_int8(T, ops, oracle, geo):
    """NITI_DSP_CONV_Int8 slot: x NHWC, w HWIO -> y NHWC + exp_out, CPU conv numerics."""
    import niti_amd
    n, ci, h, w, co, k, s, p = geo
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    rng = np.random.default_rng(206)
    x = oracle.synth_x(rng, (n, ci, h, w))
    wt, ws = oracle.synth_w(rng, (co, ci, k, k))
    y_ref, e_ref, _, _ = oracle.conv_fwd(g, x, wt, -7, ws)
    y = T.zeros((n, g.oh, g.ow, co), dtype=T.int8, device="cuda")
    e_out = i8s(T, 0)
    ex = ops.NITIExecution(niti_amd.OP_DSP_CONV_INT8, ops.conv_common(k, stride=s, pad=p))
    ins = [ops.tensor(dev(T, x.transpose(0, 2, 3, 1)), (n, ci, h, w), niti_amd.FORMAT_NHWC),
           ops.tensor(dev(T, wt.transpose(2, 3, 1, 0)), (k, k, ci, co)),
           ops.tensor(i8s(T, -7), (1, 1, 1, 1)), ops.tensor(i8s(T, ws), (1, 1, 1, 1))]
    outs = [ops.tensor(y, (n, co, g.oh, g.ow), niti_amd.FORMAT_NHWC), ops.tensor(e_out, (1, 1, 1, 1))]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    assert np.array_equal(y.cpu().numpy(), y_ref.transpose(0, 2, 3, 1))
    assert int(e_out.item()) == e_ref


@pytest.mark.parametrize("geo", [gg for gg in GEOMS if gg[2] > 1])
def test_exec_dsp_deconv_int8(T, ops, oracle, geo):
    """NITI_DSP_DECONV_Int8 slot on what grad/NITI_DSPConv_Int8_Grad.cpp:60-120 hands it: dy (stride 2:
    LeftPoolGrad-dilated to ow x ow), pad + extraPad in the common, weights
    transpose(rot180(transpose(w, {2,3,0,1})), {2,3,1,0}) and zero exponents."""
    import niti_amd
    n, ci, h, w, co, k, s, p = geo
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    rng = np.random.default_rng(207)
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    wt, _ = oracle.synth_w(rng, (co, ci, k, k))
    dx_ref, inc_ref, _, _ = oracle.conv_dgrad(g, dy, wt)
    d = dy
    if s == 2:
        ow1 = w + 2 * p - k + 1
        d = np.zeros((n, co, ow1, ow1), np.int8)
        d[:, :, ::2, ::2][:, :, :g.oh, :g.ow] = dy
    if (w - (d.shape[3] + 2 * p - k + 1)) % 2 or (h - (d.shape[2] + 2 * p - k + 1)) % 2:
        pytest.skip("reference extra-pad arithmetic undefined for this shape")
    e = (w - (d.shape[3] + 2 * p - k + 1)) // 2
    if h - (d.shape[2] + 2 * (p + e) - k + 1):
        pytest.skip("reference pads H and W by the same W-derived extra pad")
    hwio = wt.transpose(2, 3, 1, 0)                                        # forward weights [k][k][ci][co]
    wr = np.flip(hwio.transpose(2, 3, 0, 1), axis=(2, 3)).transpose(2, 3, 1, 0)  # [k][k][co][ci]
    out = T.zeros((n, h, w, ci), dtype=T.int8, device="cuda")
    e_out = i8s(T, 99)
    ex = ops.NITIExecution(niti_amd.OP_DSP_DECONV_INT8, ops.conv_common(k, stride=1, pad=p + e))
    ins = [ops.tensor(dev(T, d.transpose(0, 2, 3, 1)), (n, co, d.shape[2], d.shape[3]), niti_amd.FORMAT_NHWC),
           ops.tensor(dev(T, wr), (k, k, co, ci)), ops.tensor(i8s(T, 0), (1, 1, 1, 1)),
           ops.tensor(i8s(T, 0), (1, 1, 1, 1))]
    outs = [ops.tensor(out, (n, ci, h, w), niti_amd.FORMAT_NHWC), ops.tensor(e_out, (1, 1, 1, 1))]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    assert np.array_equal(out.cpu().numpy(), dx_ref.transpose(0, 2, 3, 1))
    assert int(e_out.item()) == inc_ref


@pytest.mark.parametrize("op", [822, 821])
@pytest.mark.parametrize("geo", GEOMS)
def test_exec_dsp_transpose_gradient_conv(T, ops, oracle, geo, op):
    """NITI_DSP_TRANSPOSEGRADIENT_CONV_Int8 / GRADIENT_SPLITBatchCONV slots
    (grad/NITI_DSPConv_Int8_Grad.cpp:160-219): {x^T = transpose(x, {3,1,2,0}), dy (stride 2:
    LeftPoolGrad-dilated to ow x ow, stride 1 in the common), 0, 0} -> dw [Ci][KH][KW][Co] + bw - 2."""
    n, ci, h, w, co, k, s, p = geo
    if s == 2 and h != w:
        pytest.skip("the graph dilates dy to a square ow x ow")
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    rng = np.random.default_rng(208)
    x = oracle.synth_x(rng, (n, ci, h, w))
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    dw_ref, bw, _, _ = oracle.conv_wgrad(g, x, dy)
    d = dy
    if s == 2:
        ow1 = w + 2 * p - k + 1
        d = np.zeros((n, co, ow1, ow1), np.int8)
        d[:, :, ::2, ::2][:, :, :g.oh, :g.ow] = dy
    xt = x.transpose(1, 2, 3, 0)                                   # NHWC x transposed {3,1,2,0}: [ci][h][w][n]
    out = T.zeros((ci, k, k, co), dtype=T.int8, device="cuda")
    e_out = i8s(T, 99)
    ex = ops.NITIExecution(op, ops.conv_common((d.shape[3], d.shape[2]), stride=1, pad=p))
    import niti_amd
    ins = [ops.tensor(dev(T, xt), (ci, n, h, w), niti_amd.FORMAT_NHWC),
           ops.tensor(dev(T, d.transpose(0, 2, 3, 1)), (n, co, d.shape[2], d.shape[3]), niti_amd.FORMAT_NHWC),
           ops.tensor(i8s(T, 0), (1, 1, 1, 1)), ops.tensor(i8s(T, 0), (1, 1, 1, 1))]
    outs = [ops.tensor(out, (ci, co, k, k), niti_amd.FORMAT_NHWC), ops.tensor(e_out, (1, 1, 1, 1))]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    assert np.array_equal(out.cpu().numpy().transpose(3, 0, 1, 2), dw_ref)
    assert int(e_out.item()) == (bw - 2 if bw else 0)


def test_exec_dsp_transpose_gradient_rejects_stride2(T, ops):
    import niti_amd
    ex = ops.NITIExecution(niti_amd.OP_DSP_TRANSPOSEGRADIENT_CONV_INT8, ops.conv_common(3, stride=2, pad=1))
    a = T.zeros((64,), dtype=T.int8, device="cuda")
    ins = [ops.tensor(a, (2, 2, 4, 4), niti_amd.FORMAT_NHWC), ops.tensor(a, (2, 2, 2, 2), niti_amd.FORMAT_NHWC)]
    outs = [ops.tensor(a, (2, 2, 3, 3), niti_amd.FORMAT_NHWC)]
    assert ex.resize(ins, outs) == 2  # NOT_SUPPORT: the graph dilates dy (LeftPoolGrad) for stride 2


@pytest.mark.parametrize("op", [801, 817, 805])
@pytest.mark.parametrize("shape", [(2, 5, 3, 7), (4, 64, 8, 8)])
def test_exec_dsp_relu_family(T, ops, oracle, op, shape):
    """NITI_DSP_RELU / NOP / RELUGRAD slots on NHWC tensors (CPU numerics)."""
    n, c, h, w = shape
    rng = np.random.default_rng(210)
    x = rng.integers(-128, 128, size=(n, h, w, c), dtype=np.int8)
    dy = rng.integers(-128, 128, size=(n, h, w, c), dtype=np.int8)
    want = {801: oracle.relu(x), 817: x, 805: oracle.relu_grad(x, dy)}[op]
    out = T.zeros((n, h, w, c), dtype=T.int8, device="cuda")
    ex = ops.NITIExecution(op, None)
    ins = [ops.tensor(dev(T, x), shape, 1)] + ([ops.tensor(dev(T, dy), shape, 1)] if op == 805 else [])
    outs = [ops.tensor(out, shape, 1)]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("geo", [(2, 20, 12, 12, 2, 2, 0), (3, 5, 9, 9, 3, 2, 1), (2, 64, 5, 5, 2, 2, 0),
                                 (1, 130, 4, 4, 2, 2, 0)])
def test_exec_dsp_maxpool_and_grad(T, ops, oracle, geo):
    """NITI_DSP_MAXPOOL (ascale passed through) and NITI_DSP_MAXPOOLGRAD slots, NHWC, first max wins."""
    n, c, h, w, k, s, p = geo
    rng = np.random.default_rng(211)
    x = rng.integers(-8, 8, size=(n, c, h, w), dtype=np.int8)  # small range: ties exercise first-max-wins
    y_ref = oracle.maxpool(x, k, s, p)
    oh, ow = y_ref.shape[2], y_ref.shape[3]
    dy = rng.integers(-128, 128, size=(n, c, oh, ow), dtype=np.int8)
    dx_ref = oracle.maxpool_grad(x, y_ref, dy, k, s, p)
    nhwc = lambda a: np.ascontiguousarray(a.transpose(0, 2, 3, 1))
    common = ops.conv_common(k, stride=s, pad=p)
    y = T.zeros((n, oh, ow, c), dtype=T.int8, device="cuda")
    sc_out = i8s(T, 0)
    ex = ops.NITIExecution(802, common)
    ins = [ops.tensor(dev(T, nhwc(x)), (n, c, h, w), 1), ops.tensor(i8s(T, -5), (1, 1, 1, 1))]
    outs = [ops.tensor(y, (n, c, oh, ow), 1), ops.tensor(sc_out, (1, 1, 1, 1))]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    assert np.array_equal(y.cpu().numpy(), nhwc(y_ref))
    assert int(sc_out.item()) == -5
    dx = T.zeros((n, h, w, c), dtype=T.int8, device="cuda")
    eg = ops.NITIExecution(807, common)
    ins = [ops.tensor(dev(T, nhwc(x)), (n, c, h, w), 1), ops.tensor(y, (n, c, oh, ow), 1),
           ops.tensor(dev(T, nhwc(dy)), (n, c, oh, ow), 1)]
    outs = [ops.tensor(dx, (n, c, h, w), 1)]
    assert eg.resize(ins, outs) == 0
    assert eg.execute(ins, outs) == 0
    assert np.array_equal(dx.cpu().numpy(), nhwc(dx_ref))


@pytest.mark.parametrize("op", [711, 804])
@pytest.mark.parametrize("batch,classes,ascale", [(7, 10, -7), (5, 10, -3), (3, 1000, -5), (2, 17, 0)])
def test_exec_loss_grad(T, ops, oracle, op, batch, classes, ascale):
    """NITI_LOSS_Grad / NITI_DSP_LOSSGRAD slots: logits, ascale, one-hot int32 target, dy -> grad."""
    rng = np.random.default_rng(212)
    logits = rng.integers(-128, 128, size=(batch, classes), dtype=np.int8)
    labels = rng.integers(0, classes, size=batch)
    onehot = np.zeros((batch, classes), np.int32)
    onehot[np.arange(batch), labels] = 1
    want = oracle.loss_grad(logits, ascale, onehot)
    out = T.zeros((batch, classes), dtype=T.int8, device="cuda")
    ex = ops.NITIExecution(op, None)
    ins = [ops.tensor(dev(T, logits), (batch, classes)), ops.tensor(i8s(T, ascale), (1, 1, 1, 1)),
           ops.tensor(dev(T, onehot), (batch, classes)), ops.tensor(dev(T, logits), (batch, classes))]
    outs = [ops.tensor(out, (batch, classes))]
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    assert np.array_equal(out.cpu().numpy(), want)


def _run_exec(ops, op, common, ins, outs):
    ex = ops.NITIExecution(op, common)
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0


def _nhwc_dims(raw):  # stored [N][H][W][C] -> logical {N, C, H, W}
    return (raw[0], raw[3], raw[1], raw[2])


@pytest.mark.parametrize("perm", [(3, 1, 2, 0), (2, 3, 0, 1), (2, 3, 1, 0), (0, 1, 2, 3)])
def test_exec_dsp_transpose(T, ops, perm):
    """NITI_DSP_TRANSPOSE on the stored axis order (the graph's transpose(x, {3,1,2,0}) etc.)."""
    rng = np.random.default_rng(213)
    x = rng.integers(-128, 128, size=(3, 5, 4, 7), dtype=np.int8)  # stored NHWC [N][H][W][C]
    want = np.ascontiguousarray(x.transpose(perm))
    out = T.zeros(want.shape, dtype=T.int8, device="cuda")
    p = T.tensor(perm, dtype=T.int32, device="cuda")
    _run_exec(ops, 808, None, [ops.tensor(dev(T, x), _nhwc_dims(x.shape), 1), ops.tensor(p, (4, 1, 1, 1))],
              [ops.tensor(out, _nhwc_dims(want.shape), 1)])
    assert np.array_equal(out.cpu().numpy(), want)


def test_exec_dsp_deconv_weight_chain(T, ops, oracle):
    """transpose(rot180(transpose(w, {2,3,0,1})), {2,3,1,0}) through the 808 / 809 slots equals the
    rotated weights the deconv slot test builds on the host (grad/NITI_DSPConv_Int8_Grad.cpp:88-92)."""
    rng = np.random.default_rng(214)
    k, ci, co = 3, 6, 10
    hwio = rng.integers(-128, 128, size=(k, k, ci, co), dtype=np.int8)
    want = np.ascontiguousarray(np.flip(hwio.transpose(2, 3, 0, 1), axis=(2, 3)).transpose(2, 3, 1, 0))
    t1 = T.zeros((ci, co, k, k), dtype=T.int8, device="cuda")
    t2 = T.zeros((ci, co, k, k), dtype=T.int8, device="cuda")
    t3 = T.zeros((k, k, co, ci), dtype=T.int8, device="cuda")
    p1 = T.tensor([2, 3, 0, 1], dtype=T.int32, device="cuda")
    p2 = T.tensor([2, 3, 1, 0], dtype=T.int32, device="cuda")
    _run_exec(ops, 808, None, [ops.tensor(dev(T, hwio), hwio.shape, 0), ops.tensor(p1, (4, 1, 1, 1))],
              [ops.tensor(t1, t1.shape, 0)])
    _run_exec(ops, 809, None, [ops.tensor(t1, t1.shape, 0)], [ops.tensor(t2, t2.shape, 0)])
    _run_exec(ops, 808, None, [ops.tensor(t2, t2.shape, 0), ops.tensor(p2, (4, 1, 1, 1))],
              [ops.tensor(t3, t3.shape, 0)])
    assert np.array_equal(t3.cpu().numpy(), want)


@pytest.mark.parametrize("op", [814, 815])
@pytest.mark.parametrize("n,c,oh,ow1", [(2, 5, 4, 7), (3, 64, 8, 16), (1, 3, 1, 2)])
def test_exec_dsp_leftpoolgrad(T, ops, op, n, c, oh, ow1):
    rng = np.random.default_rng(215)
    dy = rng.integers(-128, 128, size=(n, oh, oh, c), dtype=np.int8)
    want = np.zeros((n, ow1, ow1, c), np.int8)
    sub = want[:, ::2, ::2, :]
    m = min(oh, sub.shape[1])
    sub[:, :m, :m, :] = dy[:, :m, :m, :]
    out = T.full((n, ow1, ow1, c), 9, dtype=T.int8, device="cuda")
    _run_exec(ops, op, ops.conv_common(1, stride=2), [ops.tensor(dev(T, dy), (n, c, oh, oh), 1)],
              [ops.tensor(out, (n, c, ow1, ow1), 1)])
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("p", [0, 1, 2])
def test_exec_dsp_pad(T, ops, p):
    rng = np.random.default_rng(217)
    x = rng.integers(-128, 128, size=(2, 5, 6, 3), dtype=np.int8)
    want = np.pad(x, ((0, 0), (p, p), (p, p), (0, 0)))
    out = T.full(want.shape, 9, dtype=T.int8, device="cuda")
    _run_exec(ops, 812, ops.conv_common(1, pad=p), [ops.tensor(dev(T, x), _nhwc_dims(x.shape), 1)],
              [ops.tensor(out, _nhwc_dims(want.shape), 1)])
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("op", [803, 813])
def test_exec_dsp_reshape(T, ops, op):
    rng = np.random.default_rng(216)
    x = rng.integers(-128, 128, size=(4, 2, 2, 32), dtype=np.int8)
    out = T.zeros((4, 128), dtype=T.int8, device="cuda")
    _run_exec(ops, op, None, [ops.tensor(dev(T, x), _nhwc_dims(x.shape), 1)], [ops.tensor(out, (4, 128, 1, 1), 1)])
    assert np.array_equal(out.cpu().numpy(), x.reshape(4, 128))


@pytest.mark.parametrize("geo", [(2, 20, 12, 12, 2, 2, 0), (3, 6, 9, 9, 3, 2, 1), (4, 64, 8, 8, 2, 2, 0)])
def test_exec_cpu_pool_relu_c4(T, ops, oracle, geo):
    """The CPU graph's NITI_Relu / NITI_ReluGrad / NITI_Maxpool / NITI_PoolGrad slots (703-706) on NC4HW4."""
    n, c, h, w, k, s, p = geo
    rng = np.random.default_rng(218)
    x = rng.integers(-8, 8, size=(n, c, h, w), dtype=np.int8)
    g = rng.integers(-128, 128, size=(n, c, h, w), dtype=np.int8)
    c4 = oracle.nchw_to_c4
    dims = (n, c, h, w)
    out = T.zeros(c4(x).shape, dtype=T.int8, device="cuda")
    _run_exec(ops, 703, None, [ops.tensor(dev(T, c4(x)), dims, 2)], [ops.tensor(out, dims, 2)])
    assert np.array_equal(out.cpu().numpy(), c4(oracle.relu(x)))
    _run_exec(ops, 704, None, [ops.tensor(dev(T, c4(x)), dims, 2), ops.tensor(dev(T, c4(g)), dims, 2)],
              [ops.tensor(out, dims, 2)])
    assert np.array_equal(out.cpu().numpy(), c4(oracle.relu_grad(x, g)))
    y_ref = oracle.maxpool(x, k, s, p)
    oh, ow = y_ref.shape[2], y_ref.shape[3]
    dy = rng.integers(-128, 128, size=(n, c, oh, ow), dtype=np.int8)
    ydims = (n, c, oh, ow)
    y = T.zeros(c4(y_ref).shape, dtype=T.int8, device="cuda")
    sc = i8s(T, 0)
    common = ops.conv_common(k, stride=s, pad=p)
    _run_exec(ops, 705, common, [ops.tensor(dev(T, c4(x)), dims, 2), ops.tensor(i8s(T, 3), (1, 1, 1, 1))],
              [ops.tensor(y, ydims, 2), ops.tensor(sc, (1, 1, 1, 1))])
    assert np.array_equal(y.cpu().numpy(), c4(y_ref))
    assert int(sc.item()) == 3
    _run_exec(ops, 706, common, [ops.tensor(dev(T, c4(x)), dims, 2), ops.tensor(y, ydims, 2),
                                 ops.tensor(dev(T, c4(dy)), ydims, 2)], [ops.tensor(out, dims, 2)])
    assert np.array_equal(out.cpu().numpy(), c4(oracle.maxpool_grad(x, y_ref, dy, k, s, p)))


def test_exec_cpu_pad_and_leftpoolgrad(T, ops, oracle):
    """The CPU graph's NITI_PAD (714, NCHW) and NITI_LeftPoolGrad (718, NC4HW4): the dy the deconv gets
    (grad/NITI_Conv_Int8_Grad.cpp:101)."""
    rng = np.random.default_rng(219)
    n, c, oh, ow1, e = 3, 6, 5, 9, 1
    dy = rng.integers(-128, 128, size=(n, c, oh, oh), dtype=np.int8)
    d = np.zeros((n, c, ow1, ow1), np.int8)
    d[:, :, ::2, ::2] = dy
    c4 = oracle.nchw_to_c4
    out4 = T.full(c4(d).shape, 9, dtype=T.int8, device="cuda")
    _run_exec(ops, 718, ops.conv_common(1, stride=2), [ops.tensor(dev(T, c4(dy)), dy.shape, 2)],
              [ops.tensor(out4, d.shape, 2)])
    assert np.array_equal(out4.cpu().numpy(), c4(d))
    want = np.pad(d, ((0, 0), (0, 0), (e, e), (e, e)))
    outp = T.full(want.shape, 9, dtype=T.int8, device="cuda")
    _run_exec(ops, 714, ops.conv_common(1, pad=e), [ops.tensor(dev(T, d), d.shape, 0)], [ops.tensor(outp, want.shape, 0)])
    assert np.array_equal(outp.cpu().numpy(), want)


# --------------------------------------------------------------------------- tensor formats (§8(f)-3)
def _as_format(x_nchw, fmt, oracle):
    if fmt == 0:
        return np.ascontiguousarray(x_nchw)
    if fmt == 1:
        return np.ascontiguousarray(x_nchw.transpose(0, 2, 3, 1))
    return oracle.nchw_to_c4(x_nchw)  # MNN CPU NC4HW4 [C/4][N][H][W][4] (oracle restatement)


@pytest.mark.parametrize("shape", [(2, 5, 3, 7), (1, 8, 4, 4), (3, 1, 1, 9), (4, 130, 2, 3)])
@pytest.mark.parametrize("sf,df", [(a, b) for a in range(3) for b in range(3) if a != b])
def test_tensor_convert(T, ops, oracle, shape, sf, df):
    n, c, h, w = shape
    rng = np.random.default_rng(209)
    x = rng.integers(-128, 128, size=shape, dtype=np.int8)
    src = _as_format(x, sf, oracle)
    want = _as_format(x, df, oracle)
    d_src = dev(T, src)
    d_dst = T.full(want.shape, 77, dtype=T.int8, device="cuda")  # pad lanes must come back zero
    assert ops.convert(ops.tensor(d_src, shape, sf), ops.tensor(d_dst, shape, df)) == 0
    assert np.array_equal(d_dst.cpu().numpy(), want)


def test_tensor_convert_errors(T, ops):
    a = T.zeros(64, dtype=T.int8, device="cuda")
    b = T.zeros(64, dtype=T.int8, device="cuda")
    assert ops.convert(ops.tensor(a, (1, 4, 2, 2), 0), ops.tensor(b, (1, 4, 2, 3), 1)) == 3  # COMPUTE_SIZE_ERROR
    assert ops.convert(ops.tensor(a, (1, 4, 2, 2), 0), ops.tensor(b, (1, 4, 2, 2), 7)) == 2  # NOT_SUPPORT
    assert ops.convert(ops.tensor(a, (1, 4, 2, 2), 0), ops.tensor(a, (1, 4, 2, 2), 1)) == 5  # in place


# --------------------------------------------------------------------------- requant edge cases
@pytest.mark.parametrize("vals", [[0, 0, 0], [128, -5, 3], [200, -103, 101], [40000, -1007, 0], [1, -1, 0],
                                  [2**30, -(2**30) + 7, 12345], [127, -127, 64]])
def test_requant_act_branches(T, ops, oracle, vals):
    acc = np.zeros((1, 16), np.int32)
    acc[0, :len(vals)] = vals
    want, inc = oracle.requant_fwd(acc)
    amax = zeros_u32(T)
    a = dev(T, acc)
    ops.absmax(a, amax)
    e = i8s(T, 0)
    got = ops.requant_act(a, amax, exp_in=i8s(T, 3), wscale=i8s(T, -7), exp_out=e)
    assert np.array_equal(got.cpu().numpy(), want)
    assert int(e.item()) == int(np.int8(3 - 7 + inc))


@pytest.mark.parametrize("vals", [[0, 0], [1, -1], [2, -1], [3, -2, 1], [4, -3], [5, 7, -9],
                                  [65536, -65535, 3], [2**31 - 1, 5]])
@pytest.mark.parametrize("rule", [2, 3])
def test_requant_grad_rules(T, ops, oracle, vals, rule):
    acc = np.array(vals, np.int32)
    want, bw = (oracle.requant_wgrad if rule == 2 else oracle.requant_matmul)(acc)
    amax = zeros_u32(T)
    a = dev(T, acc)
    ops.absmax(a, amax)
    assert np.array_equal(ops.requant_grad(a, amax, rule=rule).cpu().numpy(), want)


def test_psto_all_shifts(T, ops, oracle):
    """requant_act's PSTO against the oracle for every forward shift 2..24."""
    rng = np.random.default_rng(7)
    for s in range(2, 25):
        top = 1 << (s + 7)
        acc = rng.integers(-top, top, (64, 16)).astype(np.int32)
        acc[0, 0] = min(top, 2**31 - 1)  # pin the range estimate
        want, _ = oracle.requant_fwd(acc)
        amax = zeros_u32(T)
        a = dev(T, acc)
        ops.absmax(a, amax)
        assert np.array_equal(ops.requant_act(a, amax).cpu().numpy(), want), s


# --------------------------------------------------------------------------- rest of the step
def test_pool_relu_loss_kernels(T, ops, oracle):
    rng = np.random.default_rng(301)
    for (n, c, h, w) in [(3, 20, 24, 24), (2, 52, 8, 8), (4, 64, 7, 7)]:
        y = rng.integers(-127, 128, (n, c, h, w)).astype(np.int8)
        y[rng.random(y.shape) < 0.3] = 5  # ties
        r = oracle.relu(y)
        p_ref = oracle.maxpool(r)
        r16 = ops.nchw_to_nhwc16(dev(T, r))
        p16 = ops.maxpool(r16)
        cp = r16.shape[3]
        p = p16.cpu().numpy()[..., :c].transpose(0, 3, 1, 2)
        assert np.array_equal(p, p_ref)
        dp = oracle.synth_dy(rng, p_ref.shape)
        dx_ref = oracle.relu_grad(y, oracle.maxpool_grad(r, p_ref, dp))
        dx16 = ops.maxpool_grad(r16, p16, ops.nchw_to_nhwc16(dev(T, dp)), relu=True)
        assert np.array_equal(dx16.cpu().numpy()[..., :c].transpose(0, 3, 1, 2), dx_ref)
        assert not dx16.cpu().numpy()[..., c:].any() or cp == c
        d = oracle.synth_dy(rng, y.shape)
        rg = ops.relu_grad(r16, ops.nchw_to_nhwc16(dev(T, d)))
        assert np.array_equal(rg.cpu().numpy()[..., :c].transpose(0, 3, 1, 2), oracle.relu_grad(y, d))
    for ascale in (-12, -7, -6, -3, 0, 2):
        logits = rng.integers(-127, 128, (33, 12)).astype(np.int8)
        labels = rng.integers(0, 10, 33).astype(np.int32)
        oh = np.zeros((33, 10), np.int32)
        oh[np.arange(33), labels] = 1
        want = oracle.loss_grad(logits, ascale, oh)
        lg = np.zeros((33, 16), np.int8)
        lg[:, :12] = logits
        got = ops.loss_grad(dev(T, lg), 12, i8s(T, ascale), dev(T, labels)).cpu().numpy()
        assert np.array_equal(got[:, :12], want), ascale
        assert not got[:, 12:].any()


@pytest.mark.parametrize("classes", [17, 100, 1000])
def test_loss_grad_wide_rows(T, ops, oracle, classes):
    """NITI_LOSS_Grad_Int8 over ImageNet-wide class rows (one block per sample), every ascale branch."""
    rng = np.random.default_rng(classes)
    ld = (classes + 15) // 16 * 16
    for ascale in (-12, -7, -6, -3, 0, 2):
        logits = rng.integers(-127, 128, (9, classes)).astype(np.int8)
        labels = rng.integers(0, classes, 9).astype(np.int32)
        oh = np.zeros((9, classes), np.int32)
        oh[np.arange(9), labels] = 1
        want = oracle.loss_grad(logits, ascale, oh)
        lg = np.zeros((9, ld), np.int8)
        lg[:, :classes] = logits
        got = ops.loss_grad(dev(T, lg), classes, i8s(T, ascale), dev(T, labels)).cpu().numpy()
        assert np.array_equal(got[:, :classes], want), ascale
        assert not got[:, classes:].any()


# --------------------------------------------------------------------------- full sizes
def _sample_check(acc_fn, n_samples, rng):
    for _ in range(n_samples):
        ok, got, want = acc_fn(rng)
        assert ok, (got, want)


def test_vgg11_batch256_layers_sampled(T, ops, oracle):
    """BASELINE cfg 3 sizes (batch 256): every GEMM-class op checked on 512 sampled outputs
    against exact int64 dot products, plus the split-batch linearity of the weight gradient."""
    rng = np.random.default_rng(17)
    for (ci, co, hh) in [(3, 64, 32), (256, 256, 8), (512, 512, 2)]:
        n, k, p = 256, 3, 1
        x = oracle.synth_x(rng, (n, ci, hh, hh))
        wt, _ = oracle.synth_w(rng, (co, ci, k, k))
        dy = oracle.synth_dy(rng, (n, co, hh, hh))
        gg = ops.geom(n, ci, hh, hh, co, k, pad=p)
        xp = np.pad(x, ((0, 0), (0, 0), (1, 1), (1, 1))).astype(np.int64)
        dyp = np.pad(dy, ((0, 0), (0, 0), (1, 1), (1, 1))).astype(np.int64)
        # forward
        amax = zeros_u32(T)
        acc = ops.conv_fwd_acc(gg, ops.nchw_to_nhwc16(dev(T, x)), ops.oihw_to_ohwi16(dev(T, wt)), amax).cpu().numpy()
        for _ in range(512):
            b, o, yy, xx = (int(rng.integers(0, v)) for v in (n, co, hh, hh))
            want = int((xp[b, :, yy:yy + 3, xx:xx + 3] * wt[o].astype(np.int64)).sum())
            assert acc[(b * hh + yy) * hh + xx, o] == want
        # input gradient: dx[b,c,y,x] = sum dy[b,o,y+1-ky,x+1-kx] w[o,c,ky,kx]
        w16 = ops.oihw_to_ohwi16(dev(T, wt))
        accd = ops.conv_dgrad_acc(gg, ops.nchw_to_nhwc16(dev(T, dy)), ops.ohwi16_to_ihwo16(w16, ci), amax).cpu().numpy()
        wf = wt[:, :, ::-1, ::-1].astype(np.int64)
        for _ in range(512):
            b, c, yy, xx = (int(rng.integers(0, v)) for v in (n, ci, hh, hh))
            want = int((dyp[b, :, yy:yy + 3, xx:xx + 3] * wf[:, c]).sum())
            assert accd[(b * hh + yy) * hh + xx, c] == want
        # weight gradient + linearity over the batch split
        xT = ops.nchw_to_nhwc16(dev(T, x))
        dyT = ops.nchw_to_nhwc16(dev(T, dy))
        accw = ops.conv_wgrad_acc(gg, xT, dyT).cpu().numpy()
        for _ in range(128):
            o, c, ky, kx = (int(rng.integers(0, v)) for v in (co, ci, 3, 3))
            want = int((xp[:, c, ky:ky + hh, kx:kx + hh] * dy[:, o].astype(np.int64)).sum())
            assert accw[o, ky, kx, c] == want
        g1 = ops.geom(128, ci, hh, hh, co, k, pad=p)
        a1 = ops.conv_wgrad_acc(g1, ops.nchw_to_nhwc16(dev(T, x[:128])), ops.nchw_to_nhwc16(dev(T, dy[:128])))
        a2 = ops.conv_wgrad_acc(g1, ops.nchw_to_nhwc16(dev(T, x[128:])), ops.nchw_to_nhwc16(dev(T, dy[128:])))
        assert np.array_equal((a1 + a2).cpu().numpy(), accw)


@pytest.mark.parametrize("h,ci,co,stride,relu", [(8, 64, 128, 1, True), (16, 32, 64, 1, False), (9, 48, 32, 2, True)])
def test_conv_two_phase_requant_equals_store_path(T, h, ci, co, stride, relu):
    """niti_conv_{fwd,dgrad}_phase1/2 (range, caller hook, requantise; small K recomputes the
    GEMM) give the same int8 output and exponent as the int32 accumulate + niti_requant_act path."""
    from niti_amd import ops
    rng = np.random.default_rng(h * ci + co)
    n = 3
    g = ops.geom(n, ci, h, h, co, 3, stride=stride, pad=1)
    x16 = ops.nchw_to_nhwc16(T.from_numpy(rng.integers(-127, 128, (n, ci, h, h)).astype(np.int8)).cuda())
    w = rng.integers(-127, 128, (co, ci, 3, 3)).astype(np.int8)
    w16 = ops.oihw_to_ohwi16(T.from_numpy(w).cuda())
    wT = ops.ohwi16_to_ihwo16(w16, ci)
    dy16 = ops.nchw_to_nhwc16(T.from_numpy(rng.integers(-127, 128, (n, co, g.oh, g.ow)).astype(np.int8)).cuda())
    e_in = T.tensor([-3], dtype=T.int8, device="cuda")
    ws8 = T.tensor([-6], dtype=T.int8, device="cuda")
    for op in (0, 1):
        a1, a2 = ops.new_range(), ops.new_range()
        e1, e2 = T.zeros(1, dtype=T.int8, device="cuda"), T.zeros(1, dtype=T.int8, device="cuda")
        seen = []
        if op == 0:
            acc = ops.conv_fwd_acc(g, x16, w16, a1)
            want = ops.requant_act(acc, a1, exp_in=e_in, wscale=ws8, exp_out=e1, relu=relu)
            got = ops.conv_fwd_requant(g, x16, w16, a2, exp_in=e_in, wscale=ws8, exp_out=e2, relu=relu,
                                       between=lambda a: seen.append(ops.range_max(a)))
        else:
            acc = ops.conv_dgrad_acc(g, dy16, wT, a1)
            want = ops.requant_act(acc, a1, exp_in=e_in, wscale=ws8, exp_out=e1)
            got = ops.conv_dgrad_requant(g, dy16, wT, a2, exp_in=e_in, wscale=ws8, exp_out=e2,
                                         between=lambda a: seen.append(ops.range_max(a)))
        T.cuda.synchronize()
        assert seen == [ops.range_max(a1)], op
        assert T.equal(got, want) and e1.item() == e2.item(), op


@pytest.mark.parametrize("geo", [(2, 64, 17, 17, 3, 2, 1), (3, 16, 12, 12, 3, 2, 1), (2, 32, 9, 9, 3, 1, 1),
                                 (1, 48, 10, 10, 2, 2, 0), (2, 16, 11, 11, 5, 2, 2)])
@pytest.mark.parametrize("relu", [False, True])
def test_maxpool_grad_two_pass(T, ops, oracle, geo, relu):
    """niti_maxpool_grad_ws (window first-max positions, then a gather per input pixel) equals the
    oracle's NITI_CPUPoolGrad_Int8 restatement and the one-pass kernel, ties included."""
    n, c, h, w, k, s, p = geo
    rng = np.random.default_rng(h * k + c)
    x = rng.integers(-6, 7, size=(n, c, h, w), dtype=np.int8)  # small range: many ties
    y_ref = oracle.maxpool(x, k, s, p)
    dy = rng.integers(-128, 128, size=y_ref.shape, dtype=np.int8)
    want = oracle.maxpool_grad(x, y_ref, dy, k, s, p)
    if relu:
        want = oracle.relu_grad(x, want)
    x16, y16, d16 = (ops.nchw_to_nhwc16(dev(T, a)) for a in (x, y_ref, dy))
    got2 = ops.maxpool_grad(x16, y16, d16, k, s, p, relu=relu, two_pass=True)
    got1 = ops.maxpool_grad(x16, y16, d16, k, s, p, relu=relu, two_pass=False)
    T.cuda.synchronize()
    assert T.equal(got1, got2)
    assert np.array_equal(ops.nhwc16_to_nchw(got2, c).cpu().numpy(), want)


@pytest.mark.parametrize("geo", [(2, 3, 20, 20, 7, 2, 3, 160), (1, 3, 15, 17, 3, 1, 1, 32), (3, 4, 8, 8, 3, 2, 1, 48),
                                 (2, 1, 9, 9, 5, 1, 2, 32)])
def test_im2col_small(T, ops, geo):
    """niti_im2col (the ResNet-18 stem's 1x1-over-im2col form) against a numpy im2col: column
    (ky * kw + kx) * c_in + c, zero past kh * kw * c_in and outside the image."""
    n, ci, h, w, k, s, p, kp = geo
    rng = np.random.default_rng(5)
    x = rng.integers(-127, 128, (n, ci, h, w)).astype(np.int8)
    g = ops.geom(n, ci, h, w, 8, k, stride=s, pad=p)
    got = ops.im2col(g, ops.nchw_to_nhwc16(dev(T, x)), kp).cpu().numpy()
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    xp = np.zeros((n, ci, h + 2 * p + k, w + 2 * p + k), np.int8)
    xp[:, :, p:p + h, p:p + w] = x
    ref = np.zeros((n, oh, ow, kp), np.int8)
    for ky in range(k):
        for kx in range(k):
            win = xp[:, :, ky:ky + s * oh:s, kx:kx + s * ow:s]  # [n][ci][oh][ow]
            ref[..., (ky * k + kx) * ci:(ky * k + kx + 1) * ci] = win.transpose(0, 2, 3, 1)
    assert np.array_equal(got, ref.reshape(n * oh * ow, kp))
    # the planar source (niti_im2col_nchw: the input quantiser's NCHW output)
    assert np.array_equal(ops.im2col(g, dev(T, x), kp, nchw=True).cpu().numpy(), ref.reshape(n * oh * ow, kp))


def test_conv_plan_set_forced_plans_agree(T, ops):
    """niti_conv_plan_set (the host-driven ResNet-18 step's autotuner): forced tile / K-split plans of
    the forward, input-gradient and weight-gradient GEMMs give the default plan's int32 results, with
    the workspace niti_conv_workspace_bytes reports for the forced plan."""
    rng = np.random.default_rng(8)
    n, ci, h, co = 4, 64, 14, 128
    g = ops.geom(n, ci, h, h, co, 3, stride=2, pad=1)
    x = ops.nchw_to_nhwc16(dev(T, rng.integers(-127, 128, (n, ci, h, h)).astype(np.int8)))
    dy = ops.nchw_to_nhwc16(dev(T, rng.integers(-127, 128, (n, co, g.oh, g.ow)).astype(np.int8)))
    w16 = ops.oihw_to_ohwi16(dev(T, rng.integers(-127, 128, (co, ci, 3, 3)).astype(np.int8)))
    wT = ops.ohwi16_to_ihwo16(w16, ci)
    runs = {0: lambda: ops.conv_fwd_acc(g, x, w16, zeros_u32(T)),
            1: lambda: ops.conv_dgrad_acc(g, dy, wT, zeros_u32(T)),
            2: lambda: ops.conv_wgrad_acc(g, x, dy, zeros_u32(T))}
    try:
        for op, f in runs.items():
            ops.conv_plan_set(g, op, None)
            ref = f().cpu().numpy()
            for plan in [(64, 64, 1, 0), (128, 64, 3, 2), (64, 128, 8, 2), (256, 128, 2, 2)]:
                ops.conv_plan_set(g, op, plan)
                assert np.array_equal(f().cpu().numpy(), ref), (op, plan)
    finally:
        for op in runs:
            ops.conv_plan_set(g, op, None)
