"""The paths BASELINE configs 4 and 5 time, compared with the oracle at their real sizes.

- The device input quantiser (MnistUtils.cpp:83-93) at the per-GPU ImageNet batches: 64 x 3 x 224 x
  224 (config 4) and 128 x 3 x 224 x 224 (config 5).  These shapes run the 512-block standalone
  statistics and the 2048-block grid-stride quantise loops (csrc/niti_quant.hip), which smaller
  batches never reach.  Also the model's own quantiser (its per-block statistics and the fused
  quantise + first-layer im2col) on a batch-64 VGG-16 step, with that step's first conv.
- VGG-16 at 224 px with autotuned plans and with the plans the batch-64 bench picks forced on: the
  tile-mode tap-sharing weight gradient with 128 / 64 / 32 / 16 K splits on conv1_2 .. conv3_1, and
  split-K GEMMs on the deeper layers.  Every tap of a whole step is compared with the oracle.
- Exact data parallelism where the row-segment speculative pair runs under the cross-rank MAX:
  VGG-16 at 224 px and ResNet-18 at 112 px, one image per rank through the C++ in-process group.  One rank gets an all-zero image, so its local bit width is 0 in every forward
  layer while the global one is not.  The first step has no hint, so every pair's launch B redoes
  its launch against the all-reduced max.  Every rank must equal one device stepping the whole batch.
Reference semantics: NITI_Conv_Int8.cpp:260-307 (RangeEstimate over the whole batch, then the shift
rule), NITI_DeConv_Int8.cpp:294-329, NITI_GradientConv_Int8.cpp:274-296.
"""
import ctypes as C
import os
import threading

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


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.mark.parametrize("shape", [(64, 3, 224, 224), (128, 3, 224, 224)])
def test_quantiser_at_imagenet_batches(T, shape):
    """niti_image_stats (512 blocks), niti_image_quantize NCHW and NHWC16 (2048-block grid-stride
    loops) against the oracle's exact-statistics quantiser, on the per-GPU batch of configs 4 / 5."""
    import niti_oracle as O
    from niti_amd import ops
    O.set_threads(_threads())
    rng = np.random.default_rng(shape[0])
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    d = T.from_numpy(img).cuda()
    st = ops.image_stats(d)
    assert st.cpu().numpy().astype(np.uint64).tolist() == O.image_stats(img).tolist()
    xr, ar = O.quantize_images(img)
    x, a = ops.image_quantize(d, st)
    assert int(a.item()) == ar
    assert np.array_equal(x.cpu().numpy(), xr)
    x16, a16 = ops.image_quantize_nhwc16(d, st)
    assert int(a16.item()) == ar
    x16 = x16.cpu().numpy()
    assert np.array_equal(x16[..., :3].transpose(0, 3, 1, 2), xr) and not x16[..., 3:].any()
    # data-parallel form: statistics over two halves, summed / max-ed, each half quantised with the
    # global pixel count (what the 8-GPU runs do per rank)
    h = shape[0] // 2
    s0, s1 = ops.image_stats(d[:h].contiguous()), ops.image_stats(d[h:].contiguous())
    sg = T.stack([s0[0] + s1[0], s0[1] + s1[1], T.maximum(s0[2], s1[2]), T.maximum(s0[3], s1[3])])
    x0, a0 = ops.image_quantize(d[:h].contiguous(), sg, img.size)
    x1, a1 = ops.image_quantize(d[h:].contiguous(), sg, img.size)
    assert int(a0.item()) == int(a1.item()) == ar
    assert np.array_equal(T.cat([x0, x1]).cpu().numpy(), xr)


def test_vgg16_model_quantiser_batch64(T):
    """The VGG-16 step's own input path at the bench's per-GPU batch (64 x 3 x 224 x 224): per-block
    statistics (IMAGE_STATS_SLOTS partials) and the fused quantise + conv0 im2col + conv0 range
    launch, then conv0's requantisation.  m.input() and the first conv's relu'd output against the
    oracle."""
    import niti_amd
    import niti_model_ref as R
    import niti_oracle as O
    from niti_amd.model import NitiModel
    O.set_threads(_threads())
    layers = R.vgg16_layers(224)
    W, S = R.init_weights(layers, seed=64)
    m = NitiModel(niti_amd.ARCH_VGG16, 64)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    rng = np.random.default_rng(64)
    img = rng.integers(0, 256, (64, 3, 224, 224), dtype=np.uint8)
    labels = rng.integers(0, 1000, 64).astype(np.int32)
    m.train_step_images(T.from_numpy(img).cuda(), T.from_numpy(labels).cuda())
    x, a = O.quantize_images(img)
    xd, ad = m.input()
    assert ad == a and np.array_equal(xd, x)
    g0 = O.geom(64, 3, 224, 224, 64, 3, pad=1)
    y0, _, _, _ = O.conv_fwd(g0, x, W[0], a, S[0])
    assert np.array_equal(m.tap(0, 0), O.relu(y0))
    assert m.rowconv_error() == 0


# the plans bench.py --arch vgg16 (batch 64) autotuned to in round 4 (gpurun_out/plans_vgg16_r04.json):
# (layer, phase) -> (bm, bn, splits, strategy); 32x32 = the tap-sharing weight gradient (tile mode at
# these maps), strategy 2 = split-K
VGG16_BENCH_PLANS = {
    (0, 2): (64, 64, 256, 2), (1, 2): (32, 32, 128, 2), (2, 2): (32, 32, 64, 2), (3, 2): (32, 32, 32, 2),
    (4, 2): (32, 32, 16, 2), (5, 2): (128, 128, 12, 2), (6, 2): (128, 128, 12, 2), (7, 2): (128, 128, 6, 2),
    (8, 2): (128, 128, 3, 2), (12, 2): (128, 128, 3, 2), (5, 0): (128, 128, 1, 0), (5, 1): (128, 128, 1, 0),
    (13, 0): (64, 128, 8, 2), (14, 0): (64, 64, 4, 2), (14, 1): (64, 64, 8, 2), (15, 0): (64, 64, 11, 2),
    (15, 1): (64, 64, 4, 2),
}


@pytest.mark.parametrize("plans", ["autotuned", "bench", "spec", "fused"])
def test_vgg16_224_tuned_plans_step_matches_oracle(T, plans):
    """A whole VGG-16 224-px step (batch 2) under the autotuner's plans, under the bench's batch-64
    kernel choices forced on, with every GEMM-path forward and input gradient on the speculative
    pair (plan strategy 3: launch A requantises with the previous bit width, launch B redoes it on a
    change -- no int32 tensor), or on the fused form (plan strategy 4: one launch, the accumulators
    kept in registers across the in-kernel grid barrier that carries the bit width), every tap
    against the oracle over two steps; plans dropped after."""
    import niti_amd
    from niti_amd import _lib as L
    import niti_model_ref as R
    from niti_amd._lib import NitiError
    from niti_amd.model import NitiModel
    layers = R.vgg16_layers(224)
    W, S = R.init_weights(layers, seed=31)
    rng = np.random.default_rng(31)
    m = NitiModel(niti_amd.ARCH_VGG16, 2)
    # the bench's plans also with the bench's keep_grads(False): no int8 weight-gradient copies, and
    # the pooled layers' 2x2 routes go to the next input gradient as codes (the row-segment kernels'
    # epilogues record them), their pre-pool outputs unwritten
    keep = plans != "bench"
    m.keep_grads(keep)
    try:
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
        x = rng.integers(-127, 128, (2, 3, 224, 224)).astype(np.int8)
        labels = rng.integers(0, 1000, 2).astype(np.int32)
        m.train_step(T.from_numpy(x).cuda(), -3, T.from_numpy(labels).cuda())  # fills the buffers
        if plans == "autotuned":
            m.autotune(reps=1)
        elif plans == "bench":
            for (layer, phase), p in VGG16_BENCH_PLANS.items():
                m.set_plan(layer, phase, p)
            for layer in range(1, 5):
                assert m.plan(layer, 2)[:2] == (32, 32), layer
        else:
            st = 3 if plans == "spec" else 4
            for layer in range(5, len(layers)):
                for phase in (0, 1):
                    m.set_plan(layer, phase, (128, 128, 1, st))
                    assert m.plan(layer, phase)[3] == st, (layer, phase)
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
        n0 = L.lib().niti_diag_gemm_fused_launches()
        for step in range(2):
            x = rng.integers(-127, 128, (2, 3, 224, 224)).astype(np.int8)
            labels = rng.integers(0, 1000, 2).astype(np.int32)
            m.train_step(T.from_numpy(x).cuda(), -3, T.from_numpy(labels).cuda())
            newW, rec = R.train_step(layers, W, S, x, -3, labels, classes=1000, impl="mnn", threads=_threads())
            logits, e = m.logits()
            assert e == rec["exp"][-1] and np.array_equal(logits, rec["logits"]), step
            for i in range(len(layers)):
                try:
                    fwd = m.tap(i, 0)
                except NitiError:  # (keep_grads(False): a pooled layer whose route went as codes)
                    assert not keep and layers[i]["pool"], ("fwd tap", step, i)
                    fwd = rec["r"][i]
                assert np.array_equal(fwd, rec["r"][i]), ("fwd", step, i)
                assert np.array_equal(m.tap(i, 2), rec["dy"][i]), ("dy", step, i)
                if keep:
                    assert np.array_equal(m.tap(i, 1), rec["dw"][i]), ("dw", step, i)
                assert np.array_equal(m.get_weight(i), newW[i]), ("w", step, i)
            W = newW
        assert m.rowconv_error() == 0
        if plans == "fused":
            assert L.lib().niti_diag_gemm_fused_launches() > n0
    finally:
        NitiModel.reset_plans()


def _in_threads(fns):
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001 -- re-raised in the main thread
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a rank thread hung"
    if errs:
        raise errs[0]


def _batches(rng, steps, world, per, shape, classes):
    """Per step the global int8 batch: step 0 rank 1's images all zero, step 1 random everywhere,
    step 2 rank 0's images all zero (the zero rank's forward ranges are 0, the global ones not)."""
    out = []
    for s in range(steps):
        x = rng.integers(-127, 128, (world * per,) + shape).astype(np.int8)
        zero_rank = {0: 1, 2: 0}.get(s)
        if zero_rank is not None:
            x[zero_rank * per:(zero_rank + 1) * per] = 0
        out.append((x, rng.integers(0, classes, world * per).astype(np.int32)))
    return out


def test_vgg16_224_local_dp_row_segment_pair(T):
    """VGG-16 at 224 px (the row-segment maps are 224 / 112 / 56 / 28 / 14 px, and VGG-16 inputs are
    multiples of 32), world 2, one image per rank, the C++ in-process group (the RCCL protocol's
    calls and streams): conv1_2 .. conv3_1 run the row-segment speculative pair with the MAX between
    launches A and B.  Every rank equals one full-batch device, which equals the oracle."""
    import niti_amd
    import niti_model_ref as R
    from niti_amd.model import LocalGroup, NitiModel
    world, per, hw = 2, 1, 224
    layers = R.vgg16_layers(hw)
    W, S = R.init_weights(layers, seed=112)
    full = NitiModel(niti_amd.ARCH_VGG16, world * per, hw)
    ranks = [NitiModel(niti_amd.ARCH_VGG16, per, hw) for _ in range(world)]
    group = LocalGroup(world)
    for r, m in enumerate(ranks):
        m.attach_local(group, r, exact=True)
    for m in [full] + ranks:
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
    streams = [T.cuda.Stream() for _ in range(world)]
    rng = np.random.default_rng(112)
    for step, (x, labels) in enumerate(_batches(rng, 3, world, per, (3, hw, hw), 1000)):
        full.train_step(T.from_numpy(x).cuda(), -3, T.from_numpy(labels).cuda())
        T.cuda.synchronize()
        parts = [(T.from_numpy(x[r * per:(r + 1) * per].copy()).cuda(),
                  T.from_numpy(labels[r * per:(r + 1) * per].copy()).cuda()) for r in range(world)]

        def rank_step(r):
            ranks[r].train_step(parts[r][0], -3, parts[r][1], stream=C.c_void_p(streams[r].cuda_stream))
            streams[r].synchronize()

        _in_threads([lambda r=r: rank_step(r) for r in range(world)])
        if step == 0:  # anchor the full-batch device on the oracle
            newW, rec = R.train_step(layers, W, S, x, -3, labels, classes=1000, impl="mnn", threads=_threads())
            lg, e = full.logits()
            assert e == rec["exp"][-1] and np.array_equal(lg, rec["logits"])
            for i in range(len(layers)):
                assert np.array_equal(full.tap(i, 0), rec["r"][i]), ("oracle fwd", i)
                assert np.array_equal(full.get_weight(i), newW[i]), ("oracle w", i)
        fl, fe = full.logits()
        for r, m in enumerate(ranks):
            sl = slice(r * per, (r + 1) * per)
            lg, e = m.logits()
            assert e == fe and np.array_equal(lg, fl[sl]), (step, r)
            for i in range(len(layers)):
                assert np.array_equal(m.tap(i, 0), full.tap(i, 0)[sl]), ("fwd", step, r, i)
                assert np.array_equal(m.tap(i, 2), full.tap(i, 2)[sl]), ("dy", step, r, i)
                assert np.array_equal(m.tap(i, 1), full.tap(i, 1)), ("dw", step, r, i)
                assert np.array_equal(m.get_weight(i), full.get_weight(i)), ("w", step, r, i)
    # the pairs ran: the first step's launches B redid their launch (no hint yet)
    st = ranks[1].spec_stats()
    assert sum(s[1] + s[2] for s in st[1:5]) > 0, st
    for m in [full] + ranks:
        assert m.rowconv_error() == 0


def test_resnet18_112_local_dp_row_segment_pair(T):
    """ResNet-18 at 112 px, 1000 classes, world 2 on the C++ step driver (the bench's) through the
    in-process group (the RCCL protocol's calls, order and streams): its 28 / 14-px stride-1 convs run
    the row-segment speculative pair with the MAX between A and B.  One rank's images are all zero on
    steps 0 and 2.  Every rank equals one full-batch device (every tap slice, weight gradient and
    weight), and the full-batch device equals the oracle on the first step."""
    import niti_amd
    import niti_resnet_ref as RR
    from niti_amd.model import LocalGroup, NitiModel
    world, per, hw, classes = 2, 1, 112, 1000
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=113)
    full = NitiModel(niti_amd.ARCH_RESNET18, world * per, hw, classes)
    ranks = [NitiModel(niti_amd.ARCH_RESNET18, per, hw, classes) for _ in range(world)]
    group = LocalGroup(world)
    for r, m in enumerate(ranks):
        m.attach_local(group, r, exact=True)
    for m in [full] + ranks:
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
    streams = [T.cuda.Stream() for _ in range(world)]
    rng = np.random.default_rng(113)
    for step, (x, labels) in enumerate(_batches(rng, 3, world, per, (3, hw, hw), classes)):
        full.train_step(T.from_numpy(x).cuda(), -2, T.from_numpy(labels).cuda())
        T.cuda.synchronize()
        parts = [(T.from_numpy(x[r * per:(r + 1) * per].copy()).cuda(),
                  T.from_numpy(labels[r * per:(r + 1) * per].copy()).cuda()) for r in range(world)]

        def rank_step(r):
            ranks[r].train_step(parts[r][0], -2, parts[r][1], stream=C.c_void_p(streams[r].cuda_stream))
            streams[r].synchronize()

        _in_threads([lambda r=r: rank_step(r) for r in range(world)])
        if step == 0:  # anchor the full-batch device on the oracle
            newW, rec = RR.train_step(convs, W, S, x, -2, labels, classes=classes)
            lg, e = full.logits()
            assert e == rec["exp_logits"] and np.array_equal(lg, rec["logits"])
            for i, c in enumerate(convs):
                assert np.array_equal(full.tap(i, 2), rec["dy"][i]), ("oracle dy", c["name"])
                assert np.array_equal(full.get_weight(i), newW[i]), ("oracle w", c["name"])
        fl, fe = full.logits()
        for r, m in enumerate(ranks):
            sl = slice(r * per, (r + 1) * per)
            lg, e = m.logits()
            assert e == fe and np.array_equal(lg, fl[sl]), (step, r)
            for i, c in enumerate(convs):
                assert np.array_equal(m.tap(i, 0), full.tap(i, 0)[sl]), ("fwd", step, r, c["name"])
                assert np.array_equal(m.tap(i, 2), full.tap(i, 2)[sl]), ("dy", step, r, c["name"])
                assert np.array_equal(m.tap(i, 1), full.tap(i, 1)), ("dw", step, r, c["name"])
                assert np.array_equal(m.get_weight(i), full.get_weight(i)), ("w", step, r, c["name"])
    # the pairs ran under the exchange: the first step's launches B redid theirs (no hint yet)
    assert sum(s[1] + s[2] + s[4] + s[5] for s in ranks[1].spec_stats()) > 0
    for m in [full] + ranks:
        assert m.rowconv_error() == 0
