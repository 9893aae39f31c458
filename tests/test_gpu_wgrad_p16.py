"""GPU parity of the P16 weight-gradient kernel (niti_wgrad.hip) through the C ABI.

The kernel computes NITI_GradientConv_Int8's int32 accumulator (NITI_GradientConv_Int8.cpp:165-298)
on pixel-block operands.  Checked bit for bit against the CPU oracle (small shapes) and against
the NHWC16 weight gradient, itself oracle-checked (full VGG-11 batch-256 shapes), for every split
count, plus the range word (NITI_RangeEstimate input) and repeat launches (the split-K arrival
counters must be back at zero after every launch).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def T():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import niti_amd  # noqa: F401
    return torch


@pytest.fixture(scope="module")
def ops(T):
    from niti_amd import ops
    return ops


def _dev(T, a):
    return T.from_numpy(np.ascontiguousarray(a)).to("cuda")


def _range(T, ops, amax):
    return ops.range_max(amax)


# (n, ci, h, co): 16-pixel blocks of 2 rows (8x8), 1 row (16x16), 1 image (4x4), 4 images (2x2)
SMALL = [(2, 32, 8, 32), (4, 64, 8, 32), (8, 32, 4, 64), (16, 32, 2, 32), (2, 32, 16, 64), (2, 64, 8, 60),
         (6, 96, 4, 32), (3, 32, 8, 64)]


@pytest.mark.parametrize("n,ci,h,co", SMALL)
@pytest.mark.parametrize("splits", [1, 2, 3])
def test_wgrad_p16_vs_oracle(T, ops, n, ci, h, co, splits):
    import niti_oracle as O
    rng = np.random.default_rng(n * 131 + ci + h * 7 + co + splits)
    g = O.geom(n, ci, h, h, co, 3, stride=1, pad=1)
    x = O.synth_x(rng, (n, ci, h, h))
    dy = O.synth_dy(rng, (n, co, g.oh, g.ow))
    gg = ops.geom(n, ci, h, h, co, 3, stride=1, pad=1)
    xP = ops.nhwc16_to_p16(ops.nchw_to_nhwc16(_dev(T, x)))
    dP = ops.nhwc16_to_p16(ops.nchw_to_nhwc16(_dev(T, dy)))
    amax = ops.new_range()
    acc = ops.conv_wgrad_p16_acc(gg, xP, dP, amax, splits=splits)
    ref, _ = O.conv_wgrad_acc(g, x, dy)  # [co][ci][kh][kw]
    got = acc.cpu().numpy()[:co, :, :, :ci].transpose(0, 3, 1, 2)
    assert np.array_equal(got, ref)
    assert _range(T, ops, amax) == int(np.abs(ref).max())


@pytest.mark.parametrize("layer", [(256, 128, 8, 256), (256, 256, 8, 256), (256, 256, 4, 512),
                                   (256, 512, 4, 512), (256, 512, 2, 512), (256, 64, 16, 128)])
@pytest.mark.parametrize("splits", [0, 1, 4, 8])
def test_wgrad_p16_vgg11_b256_vs_nhwc16(T, ops, layer, splits):
    n, ci, h, co = layer
    rng = np.random.default_rng(ci + co + h + splits)
    gg = ops.geom(n, ci, h, h, co, 3, stride=1, pad=1)
    x16 = _dev(T, rng.integers(-127, 128, (n, h, h, ci), dtype=np.int16).astype(np.int8))
    d16 = _dev(T, (rng.integers(-127, 128, (n, h, h, co), dtype=np.int16) *
                   (rng.random((n, h, h, co)) < 0.3)).astype(np.int8))
    a_ref = ops.new_range()
    ref = ops.conv_wgrad_acc(gg, x16, d16, a_ref)
    xP, dP = ops.nhwc16_to_p16(x16), ops.nhwc16_to_p16(d16)
    ws, _ = ops.wgrad_p16_workspace(gg, splits)
    for rep in range(2):  # the arrival counters must be zero again after a launch
        amax = ops.new_range()
        acc = ops.conv_wgrad_p16_acc(gg, xP, dP, amax, splits=splits, ws=ws)
        assert T.equal(acc, ref), (layer, splits, rep)
        assert ops.range_max(amax) == ops.range_max(a_ref)


def test_wgrad_p16_rejects_unsupported(T, ops):
    import niti_amd._lib as L
    gg = ops.geom(4, 16, 8, 8, 32, 3, stride=1, pad=1)  # Cip 16: not a whole 32-channel tile
    x = T.zeros(64, dtype=T.int8, device="cuda")
    with pytest.raises(L.NitiError):
        ops.conv_wgrad_p16_acc(gg, x, x)


@pytest.mark.parametrize("pixels,cp", [(16, 32), (48, 32), (4096, 32), (2064, 64), (1024, 128), (272, 256),
                                       (1024, 512), (80, 1024), (64, 48), (1056, 96)])
def test_nhwc16_to_p16_layout(T, ops, pixels, cp):
    """P16 [pixels/16][cp][16] is the NHWC16 [pixels][cp] tensor with each 16-pixel block transposed:
    the LDS-staged kernel (power-of-two cp, ragged last workgroup) and the generic one (48, 96)."""
    rng = np.random.default_rng(pixels + cp)
    a = rng.integers(-128, 128, (pixels, cp)).astype(np.int8)
    want = a.reshape(pixels // 16, 16, cp).transpose(0, 2, 1).copy()
    got = ops.nhwc16_to_p16(T.from_numpy(a).cuda()).cpu().numpy().reshape(pixels // 16, cp, 16)
    assert np.array_equal(got, want)
