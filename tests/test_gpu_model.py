"""GPU parity of the device-resident training step against the oracle's NITI_SGD step.

Every forward output, exponent, input gradient, int8 weight gradient and updated weight of
the step must equal the oracle (niti_model_ref.py) bit for bit, over two consecutive steps.
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


def _run(T, arch, layers, batch, steps=2, seed=5, graph=False, reuse_buffers=True, prepare=None, overlap=True,
         in_hw=0, classes=10, rowconv=True, keep_grads=True):
    """reuse_buffers: new data goes into the same device tensors every step, so with graph=True
    steps after the first replay the captured graph instead of re-capturing it.
    prepare(model, x, labels): called after one throwaway step (weights are reset after it)."""
    import niti_model_ref as R
    from niti_amd.model import NitiModel
    rng = np.random.default_rng(seed)
    W, S = R.init_weights(layers, seed=seed)
    m = NitiModel(arch, batch, in_hw)
    m.set_graph(graph)
    m.set_overlap(overlap)
    sched = rowconv if isinstance(rowconv, (list, tuple)) else [rowconv] * steps
    m.set_rowconv(sched[0])
    m.keep_grads(keep_grads)
    xd = ld = None
    l0 = layers[0]
    if prepare is not None:
        xt = T.from_numpy(rng.integers(-127, 128, (batch, l0["ci"], l0["h"], l0["h"])).astype(np.int8)).cuda()
        lt = T.from_numpy(rng.integers(0, classes, batch).astype(np.int32)).cuda()
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
        m.train_step(xt, -3, lt)
        prepare(m, xt, lt)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    for i in range(len(layers)):
        assert np.array_equal(m.get_weight(i), W[i])
    for step in range(steps):
        m.set_rowconv(sched[step])  # switching paths mid-training keeps every weight copy current
        x = rng.integers(-127, 128, (batch, l0["ci"], l0["h"], l0["h"])).astype(np.int8)
        labels = rng.integers(0, classes, batch).astype(np.int32)
        exp_in = -3
        newW, rec = R.train_step(layers, W, S, x, exp_in, labels, classes=classes)
        if xd is None or not reuse_buffers:
            xd = T.from_numpy(x).cuda()
            ld = T.from_numpy(labels).cuda()
        else:
            xd.copy_(T.from_numpy(x))
            ld.copy_(T.from_numpy(labels))
        m.train_step(xd, exp_in, ld)
        logits, e = m.logits()
        assert e == rec["exp"][-1], (step, e, rec["exp"][-1])
        assert np.array_equal(logits, rec["logits"]), step
        for i in range(len(layers)):
            if not keep_grads and layers[i]["pool"] and sched[step]:
                # keep_grads(0): a pooled layer whose 2x2 route went to the next input gradient as
                # codes (the row kernels) does not write its pre-pool output, so that tap is invalid
                from niti_amd._lib import NitiError
                try:
                    fwd = m.tap(i, 0)
                except NitiError:
                    fwd = None
                assert fwd is None or np.array_equal(fwd, rec["r"][i]), ("fwd", step, i)
            else:
                assert np.array_equal(m.tap(i, 0), rec["r"][i]), ("fwd", step, i)
            assert np.array_equal(m.tap(i, 2), rec["dy"][i]), ("dy", step, i)
            if keep_grads:
                assert np.array_equal(m.tap(i, 1), rec["dw"][i]), ("dw", step, i)
            assert np.array_equal(m.get_weight(i), newW[i]), ("w", step, i)
        W = newW
    assert m.rowconv_error() == 0  # no in-kernel grid barrier of the fused forward timed out


def test_lenet_step_matches_oracle(T):
    import niti_amd
    import niti_model_ref as R
    _run(T, niti_amd.ARCH_LENET, R.lenet_layers(), batch=64)


@pytest.mark.parametrize("graph,reuse", [(True, True), (True, False)])
def test_lenet_step_graph_replay_and_recapture(T, graph, reuse):
    import niti_amd
    import niti_model_ref as R
    _run(T, niti_amd.ARCH_LENET, R.lenet_layers(), batch=16, steps=3, seed=11, graph=graph, reuse_buffers=reuse)


def test_vgg11_step_matches_oracle(T):
    import niti_amd
    import niti_model_ref as R
    _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=8, steps=2)


def test_vgg11_step_single_stream(T):
    import niti_amd
    import niti_model_ref as R
    _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=8, steps=2, seed=6, overlap=False)


def test_vgg11_step_gemm_forward(T):
    """The LDS-staged GEMM + requantisation forward (the register-fed fused one switched off)."""
    import niti_amd
    import niti_model_ref as R
    _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=8, steps=2, seed=7, rowconv=False)


def test_vgg11_step_path_switch_no_grad_tap(T):
    """Row kernel -> GEMM passes -> row kernel across steps (the SGD kernel skips the IHWO16 copy
    while the row kernel runs the input gradient; switching back rebuilds it), and the SGD step
    without the int8 weight-gradient copy (the bench's setting)."""
    import niti_amd
    import niti_model_ref as R
    _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=8, steps=4, seed=13, rowconv=[True, False, False, True],
         keep_grads=False)


@pytest.mark.parametrize("reuse", [True, False])
def test_vgg11_step_graph_replay(T, reuse):
    """Inside a graph capture the register-fed forward runs as range + recompute launches (the fused
    launch's barrier epoch would be frozen by the capture)."""
    import niti_amd
    import niti_model_ref as R
    _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=8, steps=3, seed=12, graph=True, reuse_buffers=reuse)


def test_vgg11_ragged_batch(T):
    import niti_amd
    import niti_model_ref as R
    _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=5, steps=1, seed=9)


# Plans (tile shape, store / recompute / split-K count) change speed only: every forced plan and
# the autotuned set must still reproduce the oracle bit for bit.
PLANS = [(128, 128, 1, 0), (64, 64, 1, 1), (128, 64, 3, 2), (64, 128, 7, 2), (128, 128, 16, 2), (64, 64, 2, 2)]


@pytest.mark.parametrize("pi", range(len(PLANS)))
def test_vgg11_step_forced_plans(T, pi):
    import niti_amd
    import niti_model_ref as R
    from niti_amd.model import NitiModel

    def force(m, x, labels):
        for i in range(len(m.layers)):
            for ph in (0, 1, 2):
                if not (ph == 1 and i == 0):
                    m.set_plan(i, ph, PLANS[pi])

    try:
        _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=8, steps=1, seed=21 + pi, prepare=force)
    finally:
        NitiModel.reset_plans()


def test_vgg11_step_autotuned(T):
    import niti_amd
    import niti_model_ref as R
    from niti_amd.model import NitiModel
    seen = {}

    def tune(m, x, labels):
        m.autotune(reps=1)
        seen.update(m.plans())

    try:
        _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=8, steps=2, seed=3, prepare=tune)
    finally:
        NitiModel.reset_plans()
    assert len(seen) == 3 * 9 - 1
    # The plan contract niti_model_plan_set enforces (niti_model.hip), not which plan won the
    # timing: GEMM tiles are 64..256 wide; the tap-sharing weight-gradient kernel reports 32x32
    # and the P16 weight-gradient kernel 16x16, both unsplit (strategy 0) or split-K (strategy 2),
    # never recompute (strategy 1); the speculative pair (strategy 3) only on forward / input-gradient
    # GEMMs, unsplit; so is the fused form (strategy 4).
    for (layer, phase), (bm, bn, splits, strat) in seen.items():
        assert splits >= 1 and strat in (0, 1, 2, 3, 4), (layer, phase)
        if strat in (3, 4):
            assert phase != 2 and splits == 1, (layer, phase, splits)
        if bm in (16, 32) or bn in (16, 32):
            assert bm == bn and phase == 2 and strat in (0, 2), (layer, phase, bm, bn, strat)
            assert strat == 2 or splits == 1, (layer, phase, splits, strat)
        elif bm == 32 or bn == 32:
            assert (bm, bn) == (32, 32) and phase == 2 and strat in (0, 2), (layer, phase, bm, bn, strat)
            assert strat == 2 or splits == 1, (layer, phase, splits, strat)
        else:
            assert bm in (64, 128, 256) and bn in (64, 128, 256), (layer, phase, bm, bn)
        if phase == 2:
            assert strat != 1, (layer, phase)  # weight gradients never recompute


def test_vgg16_step_matches_oracle(T):
    """BASELINE cfg 4's network (VGG-16, 4096-4096-1000 head, 1000-class loss) at 32x32 input:
    the whole step, every tap, against the oracle."""
    import niti_amd
    import niti_model_ref as R
    _run(T, niti_amd.ARCH_VGG16, R.vgg16_layers(32), batch=2, steps=1, seed=13, in_hw=32, classes=1000)


def test_vgg16_224_step_layer_parity(T):
    """VGG-16 at ImageNet size (224x224, batch 2): one device step; the first conv's forward, the
    last conv's weight gradient (from the step's own input / dy taps) and the 1000-class loss
    gradient against the oracle."""
    import niti_amd
    import niti_model_ref as R
    import niti_oracle as O
    from niti_amd.model import NitiModel
    layers = R.vgg16_layers(224)
    W, S = R.init_weights(layers, seed=29)
    rng = np.random.default_rng(29)
    m = NitiModel(niti_amd.ARCH_VGG16, 2)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    x = rng.integers(-127, 128, (2, 3, 224, 224)).astype(np.int8)
    labels = rng.integers(0, 1000, 2).astype(np.int32)
    m.train_step(T.from_numpy(x).cuda(), -3, T.from_numpy(labels).cuda())
    g0 = O.geom(2, 3, 224, 224, 64, 3, pad=1)
    y0, _, _, _ = O.conv_fwd(g0, x, W[0], -3, S[0])
    assert np.array_equal(m.tap(0, 0), O.relu(y0))
    g12 = O.geom(2, 512, 14, 14, 512, 3, pad=1)
    dw12, _, _, _ = O.conv_wgrad(g12, m.tap(11, 0), m.tap(12, 2))
    assert np.array_equal(m.tap(12, 1), dw12)
    logits, e = m.logits()
    want = O.loss_grad(logits, e, R.onehot(labels, 1000))
    assert np.array_equal(m.tap(15, 2).reshape(2, 1000), want)


def test_vgg16_224_step_matches_oracle(T):
    """BASELINE cfg 4's per-GPU workload at ImageNet size: one whole VGG-16 step at 224x224 (batch 2,
    1000-class loss): every forward output, exponent, input gradient, int8 weight gradient and
    updated weight of all 16 layers against the oracle (its reference-structured restatement,
    exact accumulation, on every core the box gives the process).  NITI_Conv_Int8.cpp:162-310,
    NITI_GradientConv_Int8.cpp:165-298, NITI_DeConv_Int8.cpp:187-332, NITI_SGD.hpp:20-54."""
    import os

    import niti_amd
    import niti_model_ref as R
    from niti_amd.model import NitiModel
    layers = R.vgg16_layers(224)
    W, S = R.init_weights(layers, seed=29)
    rng = np.random.default_rng(29)
    m = NitiModel(niti_amd.ARCH_VGG16, 2)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    x = rng.integers(-127, 128, (2, 3, 224, 224)).astype(np.int8)
    labels = rng.integers(0, 1000, 2).astype(np.int32)
    m.train_step(T.from_numpy(x).cuda(), -3, T.from_numpy(labels).cuda())
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    newW, rec = R.train_step(layers, W, S, x, -3, labels, classes=1000, impl="mnn", threads=threads)
    logits, e = m.logits()
    assert e == rec["exp"][-1] and np.array_equal(logits, rec["logits"])
    for i in range(len(layers)):
        assert np.array_equal(m.tap(i, 0), rec["r"][i]), ("fwd", i)
        assert np.array_equal(m.tap(i, 2), rec["dy"][i]), ("dy", i)
        assert np.array_equal(m.tap(i, 1), rec["dw"][i]), ("dw", i)
        assert np.array_equal(m.get_weight(i), newW[i]), ("w", i)
    assert m.rowconv_error() == 0


@pytest.mark.parametrize("mode", [1, 2])
def test_vgg11_step_speculative_epilogue_modes(T, mode):
    """The fused row kernels' speculative epilogue (the previous launch's bit width applied while
    the grid barrier completes) must not change any result: on (1), and forced wrong on every
    launch (2: every epilogue redone with the barrier's bit width), two steps each against the
    oracle.  Off (0, the default) is what every other test runs."""
    import niti_amd
    import niti_model_ref as R
    from niti_amd import _lib as L
    lib = L.lib()
    try:
        lib.niti_diag_rowconv_speculate(mode)
        _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=32, steps=2, seed=17 + mode)
    finally:
        lib.niti_diag_rowconv_speculate(0)


@pytest.mark.parametrize("cap", [1, 3])
def test_vgg11_step_p16_copies_over_several_launches(T, cap):
    """More P16 input copies than one launch takes (the model's job cap lowered to 1 or 3): the
    step then runs the plain loss gradient and converts the inputs in several launches ahead of the
    last layer's weight gradient, instead of the fused loss + P16 launch -- two steps against the
    oracle (overlap off, the default)."""
    import niti_amd
    import niti_model_ref as R
    from niti_amd import _lib as L
    lib = L.lib()
    try:
        lib.niti_diag_p16_jobs_cap(cap)
        _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=32, steps=2, seed=41 + cap)
    finally:
        lib.niti_diag_p16_jobs_cap(0)


@pytest.mark.parametrize("batch,graph,keep", [(8, False, True), (36, False, False), (100, True, True)])
def test_vgg11_step_head_chain(T, batch, graph, keep):
    """VGG-11's classifier head as one launch (niti_head.hip: forward with the rescale, the loss
    gradient, the weight gradient and the input gradient routed through conv7's pool codes; off by
    default) at batches that leave a row tile partly empty (8, 36, 100), under graph replay too: two
    steps against the oracle, and the launch must have run."""
    import niti_amd
    import niti_model_ref as R
    from niti_amd import _lib as L
    lib = L.lib()
    n0 = lib.niti_diag_head_chain_launches()
    lib.niti_diag_head_chain(1)
    try:
        _run(T, niti_amd.ARCH_VGG11, R.vgg11_layers(), batch=batch, steps=2, seed=61 + batch, graph=graph,
             overlap=False, keep_grads=keep)
    finally:
        lib.niti_diag_head_chain(0)
    assert lib.niti_diag_head_chain_launches() > n0
