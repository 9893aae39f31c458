"""ResNet-18 (BASELINE config 5) on the C++ step driver (csrc/niti_resnet_model.hip, NITI_ARCH_RESNET18
behind the niti_model_* C ABI) against the oracle restatement oracle/niti_resnet_ref.py.

The residual / pool rules are this library's (the reference's NITI_Eltwise_Int8.cpp:20-28 is a stub),
so this parity is unpinned by construction; the convs, relu, max pool, loss gradient and NITI_SGD
follow the reference ops (NITI_Conv_Int8.cpp:162-310, NITI_GradientConv_Int8.cpp:165-298,
NITI_DeConv_Int8.cpp:187-332, NITI_SGD.hpp:20-54).  Every conv's requantised output, output gradient
and int8 weight gradient, the logits and their exponent and every updated weight must match bit for
bit; data-parallel ranks (the C++ in-process group: the RCCL path's calls, order and streams) must
equal one device running the global batch."""
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


def _model(batch, hw, classes, W, S):
    import niti_amd
    from niti_amd.model import NitiModel
    m = NitiModel(niti_amd.ARCH_RESNET18, batch, hw, classes)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    return m


def _check_step(m, convs, rec, newW, step, sl=None):
    import niti_oracle as O
    lg, e = m.logits()
    want = rec["logits"] if sl is None else rec["logits"][sl]
    assert e == rec["exp_logits"] and np.array_equal(lg, want), step
    for i, c in enumerate(convs):
        f = O.relu(rec["fwd"][i]) if m.layers[i]["relu"] else rec["fwd"][i]
        assert np.array_equal(m.tap(i, 0), f if sl is None else f[sl]), ("fwd", step, c["name"])
        assert np.array_equal(m.tap(i, 2), rec["dy"][i] if sl is None else rec["dy"][i][sl]), ("dy", step, c["name"])
        assert np.array_equal(m.tap(i, 1), rec["dw"][i]), ("dw", step, c["name"])
        assert np.array_equal(m.get_weight(i), newW[i]), ("w", step, c["name"])


@pytest.mark.parametrize("hw,batch,classes", [(32, 2, 10), (64, 3, 1000)])
def test_resnet18_cpp_step_matches_oracle(T, hw, batch, classes):
    import niti_resnet_ref as RR
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=hw + batch)
    rng = np.random.default_rng(hw * batch)
    m = _model(batch, hw, classes, W, S)
    assert [(l["c_in"], l["c_out"], l["kh"], l["stride"]) for l in m.layers] == \
        [(c["ci"], c["co"], c["k"], c["stride"]) for c in convs]
    for step in range(2):
        x = rng.integers(-127, 128, (batch, 3, hw, hw)).astype(np.int8)
        labels = rng.integers(0, classes, batch).astype(np.int32)
        newW, rec = RR.train_step(convs, W, S, x, -2, labels, classes=classes)
        m.train_step(T.from_numpy(x).cuda(), -2, T.from_numpy(labels).cuda())
        _check_step(m, convs, rec, newW, step)
        W = newW
    assert m.rowconv_error() == 0


def test_resnet18_cpp_224_images_step_matches_oracle(T):
    """BASELINE config 5's input size (224x224, batch 2, 1000 classes) from uint8 images: the
    device quantiser, the 7x7 / 2 stem over its 224-px im2col, the overlapping 3x3 / 2 max-pool
    gradient, the 56 / 28-px row-segment layers, every tap of the whole step."""
    import niti_oracle as O
    import niti_resnet_ref as RR
    O.set_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    hw, batch, classes = 224, 2, 1000
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=225)
    rng = np.random.default_rng(225)
    m = _model(batch, hw, classes, W, S)
    img = rng.integers(0, 256, (batch, 3, hw, hw)).astype(np.uint8)
    labels = rng.integers(0, classes, batch).astype(np.int32)
    x, a = O.quantize_images(img)
    newW, rec = RR.train_step(convs, W, S, x, a, labels, classes=classes)
    m.train_step_images(T.from_numpy(img).cuda(), T.from_numpy(labels).cuda())
    xd, ad = m.input()
    assert ad == a and np.array_equal(xd, x)
    _check_step(m, convs, rec, newW, 0)
    assert m.rowconv_error() == 0


def test_resnet18_cpp_224_bench_plans_without_taps(T):
    """BASELINE config 5's timed step as bench.py runs it, at 224 px on a batch of 4: the plan set the
    batch-128 bench autotuned (tests/golden/plans_resnet18_bench_r05.json, forced through set_plan:
    the stem's store plan with the requantise pass max-pooling (Pool3), the 128 / 224-split weight
    gradients, the 32x32 tap-sharing plans at 128 splits, the 2- and 8-split input gradients) and
    keep_grads(False), from uint8 images through the device quantiser.  Two steps against the oracle:
    the logits, every forward tap but the stem's (not written under Pool3 + keep_grads(False)), every
    output gradient, every new weight (NITI_Conv_Int8.cpp:260-307, NITI_GradientConv_Int8.cpp:274-296,
    NITI_SGD.hpp:20-54)."""
    import json
    import niti_oracle as O
    import niti_resnet_ref as RR
    from niti_amd._lib import NitiError
    from niti_amd.model import NitiModel
    O.set_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    hw, batch, classes = 224, 4, 1000
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=226)
    rng = np.random.default_rng(226)
    m = _model(batch, hw, classes, W, S)
    m.keep_grads(False)
    plans = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "plans_resnet18_bench_r05.json")))
    img = T.zeros((batch, 3, hw, hw), dtype=T.uint8, device="cuda")
    lab = T.zeros(batch, dtype=T.int32, device="cuda")
    try:
        m.train_step_images(img, lab)  # the bench's setup step, then its plans; the weights restored
        for k, p in plans.items():
            layer, phase = (int(v) for v in k.split(","))
            m.set_plan(layer, phase, p)
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
        # (split counts past this batch's K steps are clamped: plan_info reports the effective one)
        assert m.plan(0, 0) == (128, 64, 1, 0) and m.plan(7, 2)[:2] == (128, 64) and m.plan(7, 2)[3] == 2
        for step in range(2):
            im = rng.integers(0, 256, (batch, 3, hw, hw)).astype(np.uint8)
            lb = rng.integers(0, classes, batch).astype(np.int32)
            img.copy_(T.from_numpy(im))
            lab.copy_(T.from_numpy(lb))
            m.train_step_images(img, lab)
            x, a = O.quantize_images(im)
            newW, rec = RR.train_step(convs, W, S, x, a, lb, classes=classes)
            xd, ad = m.input()
            assert ad == a and np.array_equal(xd, x), step
            lg, e = m.logits()
            assert e == rec["exp_logits"] and np.array_equal(lg, rec["logits"]), step
            for i, c in enumerate(convs):
                if i > 0:
                    f = O.relu(rec["fwd"][i]) if m.layers[i]["relu"] else rec["fwd"][i]
                    assert np.array_equal(m.tap(i, 0), f), ("fwd", step, c["name"])
                assert np.array_equal(m.tap(i, 2), rec["dy"][i]), ("dy", step, c["name"])
                assert np.array_equal(m.get_weight(i), newW[i]), ("w", step, c["name"])
            with pytest.raises(NitiError):
                m.tap(0, 0)  # the stem's pre-pool output was never written
            W = newW
        assert m.rowconv_error() == 0
    finally:
        NitiModel.reset_plans()


def test_resnet18_cpp_autotuned_recompute_and_gemm_paths(T):
    """The autotuner's plans, then every GEMM-path forward forced onto the recompute form, then every
    GEMM-path forward and input gradient onto the fused form (plan strategy 4: one launch, the
    rescale behind the in-kernel grid barrier; 128x128 and 64x64 tiles; the strided input gradients
    keep their sub-pixel classes), then onto the speculative pair (plan strategy 3), then the row
    kernels switched off too (every conv on the GEMM pair): two steps each against the oracle; the
    plans are dropped afterwards."""
    import niti_resnet_ref as RR
    from niti_amd import _lib as L
    from niti_amd.model import NitiModel
    hw, batch, classes = 64, 3, 1000
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=78)
    rng = np.random.default_rng(78)
    m = _model(batch, hw, classes, W, S)
    try:
        x = rng.integers(-127, 128, (batch, 3, hw, hw)).astype(np.int8)
        lab = rng.integers(0, classes, batch).astype(np.int32)
        m.train_step(T.from_numpy(x).cuda(), -2, T.from_numpy(lab).cuda())
        m.autotune(reps=1)
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
        for phase in ("tuned", "recompute", "fused", "spec", "gemm"):
            if phase == "recompute":
                for i in range(len(convs)):
                    m.set_plan(i, 0, (128, 128, 1, 1))
            if phase == "fused":  # one launch with the rescale behind the grid barrier (strategy 4)
                n0 = L.lib().niti_diag_gemm_fused_launches()
                for i in range(len(convs)):
                    for ph in (0, 1):
                        m.set_plan(i, ph, (64, 64, 1, 4) if i % 2 else (128, 128, 1, 4))
            if phase == "spec":  # the speculative pair on every GEMM-path forward and input gradient
                for i in range(len(convs)):
                    for ph in (0, 1):
                        m.set_plan(i, ph, (128, 128, 1, 3))
            if phase == "gemm":  # every conv on the GEMM path (still the pair)
                m.set_rowconv(False)
            for step in range(2):
                x = rng.integers(-127, 128, (batch, 3, hw, hw)).astype(np.int8)
                lab = rng.integers(0, classes, batch).astype(np.int32)
                newW, rec = RR.train_step(convs, W, S, x, -2, lab, classes=classes)
                m.train_step(T.from_numpy(x).cuda(), -2, T.from_numpy(lab).cuda())
                _check_step(m, convs, rec, newW, (phase, step))
                W = newW
            if phase == "fused":
                assert L.lib().niti_diag_gemm_fused_launches() > n0
        assert m.rowconv_error() == 0
    finally:
        NitiModel.reset_plans()


def test_resnet18_cpp_graph_replay(T):
    """set_graph: the step captured once as a hipGraph (the speculative pairs instead of fused grid
    barriers) and replayed on new data in the same buffers: each replay equals the oracle."""
    import niti_oracle as O
    import niti_resnet_ref as RR
    hw, batch, classes = 32, 2, 10
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=79)
    rng = np.random.default_rng(79)
    m = _model(batch, hw, classes, W, S)
    m.set_graph(True)
    img = T.zeros((batch, 3, hw, hw), dtype=T.uint8, device="cuda")
    lab = T.zeros(batch, dtype=T.int32, device="cuda")
    for step in range(3):
        im = rng.integers(0, 256, (batch, 3, hw, hw)).astype(np.uint8)
        lb = rng.integers(0, classes, batch).astype(np.int32)
        img.copy_(T.from_numpy(im))
        lab.copy_(T.from_numpy(lb))
        m.train_step_images(img, lab)
        x, a = O.quantize_images(im)
        newW, rec = RR.train_step(convs, W, S, x, a, lb, classes=classes)
        _check_step(m, convs, rec, newW, step)
        W = newW


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


@pytest.mark.parametrize("world,per,hw,images,spec", [(2, 2, 32, True, False), (3, 1, 32, False, False),
                                                     (2, 1, 112, False, False), (2, 1, 112, False, True)])
def test_resnet18_cpp_local_dp_equals_full_batch(T, world, per, hw, images, spec):
    """Exact data parallelism on the C++ driver through the in-process group: `world` ranks equal
    one device stepping the whole batch (every tap slice, every weight gradient and weight) over
    three steps.  At 112 px the 28 / 14-px row-segment convs run the speculative pair with the MAX
    between its launches; int8 steps 0 and 2 give one rank all-zero images (its local forward ranges
    0, the global ones not).  spec: every GEMM-path forward / input gradient on the GEMM's speculative
    pair too (the MAX between its launches A and B)."""
    import niti_amd
    import niti_resnet_ref as RR
    from niti_amd.model import LocalGroup, NitiModel
    classes = 10
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=world * 10 + hw)
    full = _model(world * per, hw, classes, W, S)
    ranks = [NitiModel(niti_amd.ARCH_RESNET18, per, hw, classes) for _ in range(world)]
    group = LocalGroup(world)
    for r, m in enumerate(ranks):
        m.attach_local(group, r, exact=True)
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
    if spec:
        for m in (full, ranks[0]):  # plans are per GEMM shape: the full batch's and the ranks'
            for i in range(len(convs)):
                for ph in (0, 1):
                    m.set_plan(i, ph, (128, 128, 1, 3))
    streams = [T.cuda.Stream() for _ in range(world)]
    rng = np.random.default_rng(world + hw)
    try:
        _dp_steps(T, full, ranks, streams, rng, world, per, hw, classes, images, convs)
    finally:
        NitiModel.reset_plans()
    for m in [full] + ranks:
        assert m.rowconv_error() == 0
    if hw == 112:  # the pairs ran under the exchange: the first step's launches B redid theirs
        assert sum(s[1] + s[2] + s[4] + s[5] for s in ranks[0].spec_stats()) > 0


def _dp_steps(T, full, ranks, streams, rng, world, per, hw, classes, images, convs):
    for step in range(3):
        shape = (world * per, 3, hw, hw)
        lab = rng.integers(0, classes, world * per).astype(np.int32)
        if images:
            data = rng.integers(0, 256, shape).astype(np.uint8)
        else:
            data = rng.integers(-127, 128, shape).astype(np.int8)
            z = {0: world - 1, 2: 0}.get(step)
            if z is not None:
                data[z * per:(z + 1) * per] = 0
        dd, ld = T.from_numpy(data).cuda(), T.from_numpy(lab).cuda()
        if images:
            full.train_step_images(dd, ld)
        else:
            full.train_step(dd, -2, ld)
        T.cuda.synchronize()
        parts = [(dd[r * per:(r + 1) * per].contiguous(), ld[r * per:(r + 1) * per].contiguous()) for r in range(world)]

        def rank_step(r):
            s = C.c_void_p(streams[r].cuda_stream)
            if images:
                ranks[r].train_step_images(parts[r][0], parts[r][1], stream=s)
            else:
                ranks[r].train_step(parts[r][0], -2, parts[r][1], stream=s)
            streams[r].synchronize()

        _in_threads([lambda r=r: rank_step(r) for r in range(world)])
        fl, fe = full.logits()
        for r, m in enumerate(ranks):
            sl = slice(r * per, (r + 1) * per)
            lg, e = m.logits()
            assert e == fe and np.array_equal(lg, fl[sl]), (step, r)
            if images:
                xf, af = full.input()
                xr, ar = m.input()
                assert ar == af and np.array_equal(xr, xf[sl]), (step, r)
            for i, c in enumerate(convs):
                assert np.array_equal(m.tap(i, 0), full.tap(i, 0)[sl]), ("fwd", step, r, c["name"])
                assert np.array_equal(m.tap(i, 2), full.tap(i, 2)[sl]), ("dy", step, r, c["name"])
                assert np.array_equal(m.tap(i, 1), full.tap(i, 1)), ("dw", step, r, c["name"])
                assert np.array_equal(m.get_weight(i), full.get_weight(i)), ("w", step, r, c["name"])


@pytest.mark.parametrize("bias", [1, -1, 2])
def test_resnet18_cpp_gemm_pair_misses(T, bias):
    """The GEMM speculative pair (plan strategy 3 on every GEMM-path forward and input gradient) with
    launch A's guess forced off by `bias` (niti_diag_gemm_speculate): +1 / -1 make every launch B
    after the first miss (which opens the alternates' window) settle from A's alternate one bit width
    below / above, 2 makes every launch B redo the GEMM.  Three steps against the oracle each
    (NITI_Conv_Int8.cpp:260-307, NITI_DeConv_Int8.cpp:294-329)."""
    import niti_resnet_ref as RR
    from niti_amd import _lib as L
    from niti_amd.model import NitiModel
    hw, batch, classes = 64, 2, 10
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=90 + bias)
    rng = np.random.default_rng(90 + bias)
    m = _model(batch, hw, classes, W, S)
    lib = L.lib()
    try:
        for i in range(len(convs)):
            for ph in (0, 1):
                m.set_plan(i, ph, (128, 128, 1, 3))
        lib.niti_diag_gemm_speculate(bias)
        for step in range(3):
            x = rng.integers(-127, 128, (batch, 3, hw, hw)).astype(np.int8)
            lab = rng.integers(0, classes, batch).astype(np.int32)
            newW, rec = RR.train_step(convs, W, S, x, -2, lab, classes=classes)
            m.train_step(T.from_numpy(x).cuda(), -2, T.from_numpy(lab).cuda())
            _check_step(m, convs, rec, newW, step)
            W = newW
        st = m.spec_stats()
        settled = sum(s[2] + s[5] for s in st)  # GEMM pairs: misses settled from an alternate
        redone = sum(s[1] + s[4] for s in st)
        if bias == 2:
            assert redone > 0, st
        else:
            assert settled > 0, st
    finally:
        lib.niti_diag_gemm_speculate(0)
        NitiModel.reset_plans()



@pytest.mark.parametrize("plan", [(128, 128, 1, 0), (64, 64, 1, 1), (128, 64, 4, 2)])
def test_resnet18_cpp_subpix_dgrad_plans(T, plan):
    """The stride-2 input gradients (3x3 / 2 and 1x1 / 2 projections) as four sub-pixel class GEMMs
    through a row map, under a forced store / recompute / split-K plan on every input gradient
    (split-K falls back to one split per class), three steps against the oracle
    (NITI_DeConv_Int8.cpp:187-332: the transposed conv over the dilated output gradient)."""
    import niti_resnet_ref as RR
    from niti_amd.model import NitiModel
    hw, batch, classes = 64, 2, 10
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=70 + plan[3])
    rng = np.random.default_rng(70 + plan[3])
    m = _model(batch, hw, classes, W, S)
    assert any(c["stride"] == 2 and c["k"] == 3 for c in convs) and any(c["stride"] == 2 and c["k"] == 1 for c in convs)
    try:
        for i in range(1, len(convs)):
            m.set_plan(i, 1, plan)
        for step in range(3):
            x = rng.integers(-127, 128, (batch, 3, hw, hw)).astype(np.int8)
            lab = rng.integers(0, classes, batch).astype(np.int32)
            newW, rec = RR.train_step(convs, W, S, x, -2, lab, classes=classes)
            m.train_step(T.from_numpy(x).cuda(), -2, T.from_numpy(lab).cuda())
            _check_step(m, convs, rec, newW, step)
            W = newW
    finally:
        NitiModel.reset_plans()


@pytest.mark.parametrize("hw,batch,stem_plan", [(64, 3, (128, 64, 1, 0)), (112, 2, (128, 64, 1, 0)),
                                                (64, 3, (128, 64, 1, 1))])
def test_resnet18_cpp_without_debug_taps(T, hw, batch, stem_plan):
    """keep_grads(False), as bench.py steps: no int8 weight-gradient copies and, with a stem plan
    that requantises in a separate pass (strategy 0), the stem's requantise pass max-pools without
    writing its pre-pool output (Pool3); with the recompute plan (1) the pool stays its own pass.
    Every other tap, the logits and the new weights still equal the oracle's; the weight-gradient
    taps, and the stem's forward tap when fused, report NITI_INVALID_VALUE."""
    import niti_resnet_ref as RR
    import niti_oracle as O
    from niti_amd._lib import NitiError
    from niti_amd.model import NitiModel
    convs = RR.resnet18_convs(hw, 1000)
    W, S = RR.init_weights(convs, seed=hw + 7)
    rng = np.random.default_rng(hw + 7)
    m = _model(batch, hw, 1000, W, S)
    m.keep_grads(False)
    m.set_plan(0, 0, stem_plan)
    try:
        _steps_without_taps(T, m, RR, O, NitiError, convs, W, S, rng, batch, hw, stem_plan[3] == 0)
    finally:
        NitiModel.reset_plans()


def _steps_without_taps(T, m, RR, O, NitiError, convs, W, S, rng, batch, hw, fused):
    for step in range(2):
        x = rng.integers(-127, 128, (batch, 3, hw, hw)).astype(np.int8)
        lab = rng.integers(0, 1000, batch).astype(np.int32)
        newW, rec = RR.train_step(convs, W, S, x, -2, lab, classes=1000)
        m.train_step(T.from_numpy(x).cuda(), -2, T.from_numpy(lab).cuda())
        lg, e = m.logits()
        assert e == rec["exp_logits"] and np.array_equal(lg, rec["logits"]), step
        for i, c in enumerate(convs):
            if i > 0:
                f = O.relu(rec["fwd"][i]) if m.layers[i]["relu"] else rec["fwd"][i]
                assert np.array_equal(m.tap(i, 0), f), ("fwd", step, c["name"])
            assert np.array_equal(m.tap(i, 2), rec["dy"][i]), ("dy", step, c["name"])
            assert np.array_equal(m.get_weight(i), newW[i]), ("w", step, c["name"])
        if fused:
            with pytest.raises(NitiError):
                m.tap(0, 0)
        else:
            assert np.array_equal(m.tap(0, 0), O.relu(rec["fwd"][0])), ("fwd", step, "stem")
        with pytest.raises(NitiError):
            m.tap(1, 1)
        W = newW
    assert m.rowconv_error() == 0
