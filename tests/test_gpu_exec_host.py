"""The drop-in boundary with HOST tensors, as MNN's CPU backend hands them to an Execution.

The reference's demo pins MNN_FORWARD_CPU (MnistUtils.cpp:43), so every Execution receives
Tensor::host<T>() pointers (source/core/Execution.hpp:24-82, express/Executor.cpp:559-569).
niti_execution_execute stages any non-device tensor through device buffers and returns once the
host outputs are written, so the CPU-creator adapter of INTEGRATION.md works unchanged.  Here the
conv, deconv, gradient-conv, matmul, loss-gradient and transpose Executions run on pageable host
(CPU torch) tensors and must equal the oracle bit for bit, and mixed host/device inputs work.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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


def host(T, a):
    """A pageable host tensor (what Tensor::host<T>() is on the CPU backend)."""
    return T.from_numpy(np.ascontiguousarray(a).copy())


def _run(ops, op, common, ins, outs):
    ex = ops.NITIExecution(op, common)
    assert ex.resize(ins, outs) == 0
    assert ex.execute(ins, outs) == 0
    return ex


@pytest.mark.parametrize("geo", [(3, 3, 16, 16, 64, 3, 1, 1), (2, 64, 8, 8, 128, 3, 1, 1), (5, 6, 9, 9, 8, 3, 2, 1),
                                 (4, 20, 12, 12, 52, 5, 1, 0)])
def test_host_conv_int8(T, ops, oracle, geo):
    import niti_amd
    n, ci, h, w, co, k, s, p = geo
    rng = np.random.default_rng(301)
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    x = oracle.synth_x(rng, (n, ci, h, w))
    wt, ws = oracle.synth_w(rng, (co, ci, k, k))
    _, e_ref, y4_ref = oracle.mnn_conv_fwd(g, x, wt, -7, ws)
    y4 = T.zeros(y4_ref.shape, dtype=T.int8)
    e_out = T.zeros(1, dtype=T.int8)
    ins = [ops.tensor(host(T, oracle.nchw_to_c4(x)), (n, ci, h, w), niti_amd.FORMAT_NC4HW4),
           ops.tensor(host(T, wt), (co, ci, k, k)), ops.tensor(T.tensor([-7], dtype=T.int8), (1, 1, 1, 1)),
           ops.tensor(T.tensor([ws], dtype=T.int8), (1, 1, 1, 1))]
    outs = [ops.tensor(y4, (n, co, g.oh, g.ow), niti_amd.FORMAT_NC4HW4), ops.tensor(e_out, (1, 1, 1, 1))]
    _run(ops, niti_amd.OP_CONV_INT8, ops.conv_common(k, stride=s, pad=p, input_count=ci, output_count=co), ins, outs)
    assert np.array_equal(y4.numpy(), y4_ref)
    assert int(e_out.item()) == e_ref


def test_host_conv_int8_mixed_and_repeated(T, ops, oracle):
    """Host activations with device weights; the staging buffers are reused by a second execute
    with new host data."""
    import niti_amd
    n, ci, h, w, co, k = 2, 16, 8, 8, 32, 3
    g = oracle.geom(n, ci, h, w, co, k, stride=1, pad=1)
    rng = np.random.default_rng(302)
    wt, ws = oracle.synth_w(rng, (co, ci, k, k))
    ex = ops.NITIExecution(niti_amd.OP_CONV_INT8, ops.conv_common(k, stride=1, pad=1, input_count=ci,
                                                                  output_count=co))
    wd = T.from_numpy(wt).cuda()
    for _ in range(2):
        x = oracle.synth_x(rng, (n, ci, h, w))
        _, e_ref, y4_ref = oracle.mnn_conv_fwd(g, x, wt, -5, ws)
        y4 = T.zeros(y4_ref.shape, dtype=T.int8)
        e_out = T.zeros(1, dtype=T.int8)
        ins = [ops.tensor(host(T, oracle.nchw_to_c4(x)), (n, ci, h, w), 2), ops.tensor(wd, (co, ci, k, k)),
               ops.tensor(T.tensor([-5], dtype=T.int8), (1, 1, 1, 1)),
               ops.tensor(T.tensor([ws], dtype=T.int8, device="cuda"), (1, 1, 1, 1))]
        outs = [ops.tensor(y4, (n, co, g.oh, g.ow), 2), ops.tensor(e_out, (1, 1, 1, 1))]
        assert ex.resize(ins, outs) == 0
        assert ex.execute(ins, outs) == 0
        assert np.array_equal(y4.numpy(), y4_ref) and int(e_out.item()) == e_ref


@pytest.mark.parametrize("geo", [(3, 8, 8, 8, 12, 3, 1, 1), (2, 64, 8, 8, 128, 3, 1, 1)])
def test_host_deconv_int8(T, ops, oracle, geo):
    import niti_amd
    n, ci, h, w, co, k, s, p = geo
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    rng = np.random.default_rng(303)
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    wt, _ = oracle.synth_w(rng, (co, ci, k, k))
    dx_ref, _, _ = oracle.mnn_conv_dgrad(g, dy, wt)
    e = (w - (dy.shape[3] + 2 * p - k + 1)) // 2
    d = np.pad(dy, ((0, 0), (0, 0), (e, e), (e, e))) if e else dy
    out4 = T.zeros(((ci + 3) // 4, n, h, w, 4), dtype=T.int8)
    ins = [ops.tensor(host(T, oracle.nchw_to_c4(d)), (n, co, d.shape[2], d.shape[3]), 2),
           ops.tensor(host(T, wt.transpose(1, 0, 2, 3)), (ci, co, k, k))]
    outs = [ops.tensor(out4, (n, ci, h, w), 2)]
    _run(ops, niti_amd.OP_DECONV_INT8, ops.conv_common(k, stride=1, pad=p, input_count=co, output_count=ci), ins, outs)
    assert np.array_equal(oracle.c4_to_nchw(out4.numpy(), ci), dx_ref)


@pytest.mark.parametrize("geo", [(3, 3, 16, 16, 64, 3, 1, 1), (2, 64, 8, 8, 128, 3, 1, 1)])
def test_host_gradient_conv_int8(T, ops, oracle, geo):
    import niti_amd
    n, ci, h, w, co, k, s, p = geo
    g = oracle.geom(n, ci, h, w, co, k, stride=s, pad=p)
    rng = np.random.default_rng(304)
    x = oracle.synth_x(rng, (n, ci, h, w))
    dy = oracle.synth_dy(rng, (n, co, g.oh, g.ow))
    dw_ref, _, _ = oracle.mnn_conv_wgrad(g, x, dy)
    xT4 = oracle.nchw_to_c4(np.ascontiguousarray(x.transpose(1, 0, 2, 3)))
    dyT = np.ascontiguousarray(dy.transpose(1, 0, 2, 3))
    out4 = T.zeros(((co + 3) // 4, ci, k, k, 4), dtype=T.int8)
    ins = [ops.tensor(host(T, xT4), (ci, n, h, w), 2), ops.tensor(host(T, dyT), (co, n, g.oh, g.ow))]
    outs = [ops.tensor(out4, (ci, co, k, k), 2)]
    _run(ops, niti_amd.OP_GRADIENT_CONV_INT8,
         ops.conv_common((g.ow, g.oh), stride=1, pad=p, input_count=n, output_count=co), ins, outs)
    assert np.array_equal(oracle.c4_to_nchw(out4.numpy(), co).transpose(1, 0, 2, 3), dw_ref)


def test_host_matmul_int8(T, ops, oracle):
    import niti_amd
    rng = np.random.default_rng(305)
    m, o, k = 500, 12, 64
    B = oracle.synth_x(rng, (m, k))
    A = oracle.synth_dy(rng, (o, k))
    want, _, _, _ = oracle.matmul(B, A)
    out = T.zeros((m, o), dtype=T.int8)
    _run(ops, niti_amd.OP_MATMUL_INT8, None, [ops.tensor(host(T, B), (m, k)), ops.tensor(host(T, A), (o, k))],
         [ops.tensor(out, (m, o))])
    assert np.array_equal(out.numpy().T, want)


@pytest.mark.parametrize("op", [711, 804])
def test_host_loss_grad(T, ops, oracle, op):
    """The int32 one-hot target is staged at its own element size."""
    rng = np.random.default_rng(306)
    batch, classes, ascale = 9, 10, -6
    logits = rng.integers(-128, 128, size=(batch, classes), dtype=np.int8)
    onehot = np.zeros((batch, classes), np.int32)
    onehot[np.arange(batch), rng.integers(0, classes, size=batch)] = 1
    want = oracle.loss_grad(logits, ascale, onehot)
    out = T.zeros((batch, classes), dtype=T.int8)
    ins = [ops.tensor(host(T, logits), (batch, classes)), ops.tensor(T.tensor([ascale], dtype=T.int8), (1, 1, 1, 1)),
           ops.tensor(host(T, onehot), (batch, classes)), ops.tensor(host(T, logits), (batch, classes))]
    _run(ops, op, None, ins, [ops.tensor(out, (batch, classes))])
    assert np.array_equal(out.numpy(), want)


def test_host_dsp_transpose(T, ops):
    rng = np.random.default_rng(307)
    x = rng.integers(-128, 128, size=(3, 5, 4, 7), dtype=np.int8)
    perm = (3, 1, 2, 0)
    want = np.ascontiguousarray(x.transpose(perm))
    out = T.zeros(want.shape, dtype=T.int8)
    nd = lambda s: (s[0], s[3], s[1], s[2])  # noqa: E731
    _run(ops, 808, None, [ops.tensor(host(T, x), nd(x.shape), 1), ops.tensor(T.tensor(perm, dtype=T.int32), (4, 1, 1, 1))],
         [ops.tensor(out, nd(want.shape), 1)])
    assert np.array_equal(out.numpy(), want)


@pytest.mark.parametrize("shape,k,s", [((4, 8, 8, 32), 2, 2), ((6, 4, 4, 64), 2, 2), ((5, 6, 6, 40), 2, 3),
                                       ((3, 9, 9, 48), 3, 3)])
def test_dsp_maxpool_grad_ref_806(T, ops, oracle, shape, k, s):
    """Slot 806 (NITI_DSPMaxPoolGradRef_Int8.cpp:17-80) on device tensors against the oracle's loop
    restatement: its [batch][height][width * channel] reading, its y / dy index and the bytes it
    leaves untouched (output pre-filled with a marker)."""
    rng = np.random.default_rng(308 + k + s)
    n, h, w, c = shape
    x = rng.integers(-4, 4, size=shape, dtype=np.int8)           # ties exercise the first-match rule
    ylen = max(n * h * w * c // (k * k), 1) + 1024
    y = rng.integers(-4, 4, size=ylen, dtype=np.int8)
    y[: x.size // (k * k)] = x.reshape(-1)[::k * k][: x.size // (k * k)]  # many exact matches
    dy = rng.integers(-127, 128, size=ylen, dtype=np.int8)
    init = np.full(shape, 77, np.int8)
    want = oracle.maxpool_grad_ref806(x, y, dy, init, k, k, s, s)
    out = T.from_numpy(init.copy()).cuda()
    nd = (n, c, h, w)
    _run(ops, 806, ops.conv_common(k, stride=s),
         [ops.tensor(T.from_numpy(x).cuda(), nd, 1), ops.tensor(T.from_numpy(y).cuda(), (ylen, 1, 1, 1), 1),
          ops.tensor(T.from_numpy(dy).cuda(), (ylen, 1, 1, 1), 1)], [ops.tensor(out, nd, 1)])
    assert np.array_equal(out.cpu().numpy(), want)


def test_dsp_maxpool_grad_ref_806_rejects_overlap(T, ops):
    x = T.zeros((2, 4, 4, 128), dtype=T.int8, device="cuda")
    ex = ops.NITIExecution(806, ops.conv_common(3, stride=2))
    t = ops.tensor(x, (2, 128, 4, 4), 1)
    assert ex.resize([t, t, t], [t]) == 2  # NOT_SUPPORT: stride < kernel (order-dependent in the reference)


@pytest.mark.parametrize("op_name", ["conv", "deconv"])
def test_fused_barrier_timeout_returns_no_execution(T, ops, oracle, op_name):
    """A fused row-kernel launch whose grid barrier times out (forced: the barrier waits for one
    arrival that never comes, with a short poll limit) flags its results invalid: a synchronous
    host-tensor call returns NITI_NO_EXECUTION (ErrorCode.hpp:17-30) instead of NO_ERROR, the
    asynchronous device-tensor path reports it through niti_execution_status, and once the knob is
    reset the same handle computes the oracle's result again."""
    import niti_amd
    from niti_amd import _lib as L
    n, ci, h, co, k = 16, 64, 8, 64, 3
    rng = np.random.default_rng(311)
    g = oracle.geom(n, ci, h, h, co, k, stride=1, pad=1)
    x = oracle.synth_x(rng, (n, ci, h, h))
    wt, ws = oracle.synth_w(rng, (co, ci, k, k))
    _, e_ref, y4_ref = oracle.mnn_conv_fwd(g, x, wt, -7, ws)
    op = niti_amd.OP_CONV_INT8 if op_name == "conv" else niti_amd.OP_DECONV_INT8
    ex = ops.NITIExecution(op, ops.conv_common(k, stride=1, pad=1, input_count=ci, output_count=co))

    def io(dev):
        mk = (lambda a: T.from_numpy(np.ascontiguousarray(a)).cuda()) if dev else (lambda a: host(T, a))
        y4 = T.zeros(y4_ref.shape, dtype=T.int8, device="cuda" if dev else "cpu")
        ins = [ops.tensor(mk(oracle.nchw_to_c4(x)), (n, ci, h, h), niti_amd.FORMAT_NC4HW4),
               ops.tensor(mk(wt), (co, ci, k, k))]
        outs = [ops.tensor(y4, (n, co, h, h), niti_amd.FORMAT_NC4HW4)]
        if op_name == "conv":
            e_out = T.zeros(1, dtype=T.int8, device=y4.device)
            ins += [ops.tensor(mk(np.array([-7], np.int8)), (1, 1, 1, 1)), ops.tensor(mk(np.array([ws], np.int8)), (1, 1, 1, 1))]
            outs.append(ops.tensor(e_out, (1, 1, 1, 1)))
        return ins, outs, y4

    ins, outs, y4 = io(False)
    assert ex.resize(ins, outs) == 0
    lib = L.lib()
    try:
        lib.niti_diag_rowconv_barrier(2000, 1)
        assert ex.execute(ins, outs) == 4            # host tensors: synchronous, NO_EXECUTION
        ins_d, outs_d, _ = io(True)
        assert ex.execute(ins_d, outs_d) == 0         # device tensors: asynchronous launch
        assert ex.status() == 4                       # ... and its status
        assert ex.status() == 0                       # the flag was cleared
    finally:
        lib.niti_diag_rowconv_barrier(0, 0)
    assert ex.execute(ins, outs) == 0
    if op_name == "conv":
        assert np.array_equal(y4.numpy(), y4_ref)


def test_model_step_reports_barrier_timeout(T):
    """The whole-step driver: a forced barrier timeout in the fused row kernels is visible through
    niti_model_rowconv_error (bench.py asserts it is 0 after its timed and isolated regions)."""
    import niti_amd
    import niti_model_ref as R
    from niti_amd import _lib as L
    from niti_amd.model import NitiModel
    layers = R.vgg11_layers()
    W, S = R.init_weights(layers, seed=5)
    m = NitiModel(niti_amd.ARCH_VGG11, 32)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    rng = np.random.default_rng(5)
    img = T.from_numpy(rng.integers(0, 256, (32, 3, 32, 32)).astype(np.uint8)).cuda()
    lab = T.from_numpy(rng.integers(0, 10, 32).astype(np.int32)).cuda()
    m.train_step_images(img, lab)
    assert m.rowconv_error() == 0
    lib = L.lib()
    try:
        lib.niti_diag_rowconv_barrier(2000, 1)
        m.train_step_images(img, lab)
        T.cuda.synchronize()
    finally:
        lib.niti_diag_rowconv_barrier(0, 0)
    assert m.rowconv_error() == 1
