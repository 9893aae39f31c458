"""ResNet-18's residual ops on their own, through the split device API (niti_amd.ops over the C ABI):
the exponent-aligned residual add, its fused range + requantise form, the global sum pool and its
broadcast gradient, against oracle/niti_resnet_ref.py.

The reference has no residual rule (NITI_Eltwise_Int8.cpp:20-28 is an empty stub), so these rules
are this library's and their parity is unpinned by construction.  Whole ResNet-18 steps run on the
C++ step driver (tests/test_gpu_resnet_cpp.py)."""
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


def test_residual_add_and_sum_pool(T):
    """The two new kernels alone: exponent gaps 0..30 (the 23-bit cap and the floor shift of the
    low operand), and the sum pool with its broadcast gradient."""
    import niti_resnet_ref as RR
    from niti_amd import ops
    rng = np.random.default_rng(7)
    a = rng.integers(-128, 128, (4, 5, 5, 32)).astype(np.int8)
    b = rng.integers(-128, 128, (4, 5, 5, 32)).astype(np.int8)
    for ea, eb in [(0, 0), (3, -2), (-5, 4), (10, -20), (-30, 0), (7, 7)]:
        amax = ops.new_range()
        z, ez = ops.residual_add(T.from_numpy(a).cuda(), T.tensor([ea], dtype=T.int8, device="cuda"),
                                 T.from_numpy(b).cuda(), T.tensor([eb], dtype=T.int8, device="cuda"), amax)
        zr, ezr = RR.residual_add(a, ea, b, eb)
        assert np.array_equal(z.cpu().numpy(), zr) and int(ez.item()) == ezr, (ea, eb)
        assert ops.range_max(amax) == int(np.abs(zr.astype(np.int64)).max())
    x = rng.integers(-128, 128, (3, 7, 7, 48)).astype(np.int8)
    amax = ops.new_range()
    acc = ops.sum_pool(T.from_numpy(x).cuda(), amax).cpu().numpy()
    assert np.array_equal(acc, x.astype(np.int32).sum(axis=(1, 2)))
    assert ops.range_max(amax) == int(np.abs(acc).max())
    dy = rng.integers(-128, 128, (3, 48)).astype(np.int8)
    dx = ops.sum_pool_grad(T.from_numpy(dy).cuda(), 7, 7).cpu().numpy()
    assert np.array_equal(dx, np.broadcast_to(dy[:, None, None, :], (3, 7, 7, 48)))


def test_residual_requant_fused_equals_two_pass(T):
    """The fused residual requantisation (range pass without z, then z recomputed while
    requantising) equals niti_residual_add + niti_requant_act on the stored z: every exponent gap
    0..30, relu on and off."""
    from niti_amd import ops
    rng = np.random.default_rng(11)
    n = 4096
    for gap in list(range(0, 31, 3)) + [23, 24]:
        for relu in (False, True):
            a = T.from_numpy(rng.integers(-127, 128, n).astype(np.int8)).cuda()
            b = T.from_numpy(rng.integers(-127, 128, n).astype(np.int8)).cuda()
            ea = T.tensor([-5], dtype=T.int8, device="cuda")
            eb = T.tensor([-5 - gap if gap % 2 else -5 + gap], dtype=T.int8, device="cuda")
            a1, a2 = ops.new_range(), ops.new_range()
            z, ez1 = ops.residual_add(a, ea, b, eb, a1)
            e1 = T.zeros(1, dtype=T.int8, device="cuda")
            want = ops.requant_act(z.view(-1, 16), a1, exp_in=ez1, exp_out=e1, relu=relu).view(-1)
            ops.residual_range(a, ea, b, eb, a2)
            got, ez2, e2 = ops.residual_requant(a, ea, b, eb, a2, relu=relu)
            T.cuda.synchronize()
            assert ops.range_max(a1) == ops.range_max(a2), gap
            assert T.equal(got, want) and ez1.item() == ez2.item() and e1.item() == e2.item(), (gap, relu)
