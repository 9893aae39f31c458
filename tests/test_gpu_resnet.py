"""ResNet-18 (BASELINE config 5) NITI step on the HIP ops against the oracle restatement.

The reference has no ResNet NITI model and no residual rule (NITI_Eltwise_Int8.cpp:20-28 is an
empty stub); oracle/niti_resnet_ref.py states the rules this library uses (exponent-aligned
residual add and gradient sum, global sum pool, gradient exponents), so this parity is unpinned by
construction.  Everything else -- the 7x7 / 2 stem, the 3x3 / 2 max pool, stride-2 3x3 and 1x1
projection convs and their input / weight gradients, the 1000-way head, NITI_SGD -- follows the
reference ops and must match bit for bit: every conv's requantised output, output gradient and
int8 weight gradient, the logits and their exponent, and the updated weights, over two steps."""
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


@pytest.mark.parametrize("hw,batch,classes", [(32, 2, 10), (64, 3, 1000)])
def test_resnet18_step_matches_oracle(T, hw, batch, classes):
    import niti_oracle as O
    import niti_resnet_ref as RR
    from niti_amd.resnet import ResNet18
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=hw + batch)
    rng = np.random.default_rng(hw * batch)
    m = ResNet18(batch, hw, classes)
    assert [c["name"] for c in m.convs] == [c["name"] for c in convs]
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    m.record = True
    for step in range(2):
        x = rng.integers(-127, 128, (batch, 3, hw, hw)).astype(np.int8)
        labels = rng.integers(0, classes, batch).astype(np.int32)
        newW, rec = RR.train_step(convs, W, S, x, -2, labels, classes=classes)
        m.train_step(T.from_numpy(x).cuda(), -2, T.from_numpy(labels).cuda())
        t = m.taps()
        assert t["exp_logits"] == rec["exp_logits"] and np.array_equal(t["logits"], rec["logits"]), step
        for i, c in enumerate(convs):
            relu = m.rec["fwd"][i][1]
            want = O.relu(rec["fwd"][i]) if relu else rec["fwd"][i]
            assert np.array_equal(t["fwd"][i], want), ("fwd", step, c["name"])
            assert np.array_equal(t["dy"][i], rec["dy"][i]), ("dy", step, c["name"])
            assert np.array_equal(t["dw"][i], rec["dw"][i]), ("dw", step, c["name"])
            assert np.array_equal(m.get_weight(i), newW[i]), ("w", step, c["name"])
        W = newW


def test_resnet18_autotuned_and_recompute_forwards_match_oracle(T):
    """The autotuner's per-shape plans, then every GEMM-path forward forced onto the two-phase
    recompute form (strategy 1: range pass, GEMM recomputed and requantised -- what the autotuner
    picks for the stem), two steps against the oracle; the plans are cleared afterwards."""
    import niti_oracle as O
    import niti_resnet_ref as RR
    from niti_amd import ops
    from niti_amd.resnet import ResNet18
    hw, batch, classes = 64, 3, 1000
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=77)
    rng = np.random.default_rng(77)
    m = ResNet18(batch, hw, classes)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    try:
        m.autotune(reps=1)
        for i in range(len(m.convs)):
            if not (m.use_rows and m.rows[i]):
                ops.conv_plan_set(m.geoms[i], 0, (128, 128, 1, 1))
                m.fwd_recompute.add(m._fwd_key(i))
        m.record = True
        for step in range(2):
            x = rng.integers(-127, 128, (batch, 3, hw, hw)).astype(np.int8)
            labels = rng.integers(0, classes, batch).astype(np.int32)
            newW, rec = RR.train_step(convs, W, S, x, -2, labels, classes=classes)
            m.train_step(T.from_numpy(x).cuda(), -2, T.from_numpy(labels).cuda())
            t = m.taps()
            assert t["exp_logits"] == rec["exp_logits"] and np.array_equal(t["logits"], rec["logits"]), step
            for i, c in enumerate(convs):
                relu = m.rec["fwd"][i][1]
                want = O.relu(rec["fwd"][i]) if relu else rec["fwd"][i]
                assert np.array_equal(t["fwd"][i], want), ("fwd", step, c["name"])
                assert np.array_equal(t["dy"][i], rec["dy"][i]), ("dy", step, c["name"])
                assert np.array_equal(t["dw"][i], rec["dw"][i]), ("dw", step, c["name"])
                assert np.array_equal(m.get_weight(i), newW[i]), ("w", step, c["name"])
            W = newW
    finally:
        for g in m.geoms:
            for op in (0, 1, 2):
                ops.conv_plan_set(g, op, None)


def test_resnet18_224_step_matches_oracle(T):
    """BASELINE config 5's input size (224x224, batch 2, 1000 classes), one whole step against the
    oracle: the 7x7 / 2 stem and its weight gradient over the 224-px input, the overlapping 3x3 / 2
    max-pool gradient 112 -> 56 (the two-pass workspace kernel), the 56x56 stage's weight gradients
    (the per-lane K-major loader) and every other tap, bit for bit."""
    import niti_oracle as O
    import niti_resnet_ref as RR
    from niti_amd.resnet import ResNet18
    O.set_threads(16)
    hw, batch, classes = 224, 2, 1000
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=224)
    rng = np.random.default_rng(224)
    m = ResNet18(batch, hw, classes)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    m.record = True
    x = rng.integers(-127, 128, (batch, 3, hw, hw)).astype(np.int8)
    labels = rng.integers(0, classes, batch).astype(np.int32)
    newW, rec = RR.train_step(convs, W, S, x, -2, labels, classes=classes)
    m.train_step(T.from_numpy(x).cuda(), -2, T.from_numpy(labels).cuda())
    t = m.taps()
    assert t["exp_logits"] == rec["exp_logits"] and np.array_equal(t["logits"], rec["logits"])
    for i, c in enumerate(convs):
        relu = m.rec["fwd"][i][1]
        want = O.relu(rec["fwd"][i]) if relu else rec["fwd"][i]
        assert np.array_equal(t["fwd"][i], want), ("fwd", c["name"])
        assert np.array_equal(t["dy"][i], rec["dy"][i]), ("dy", c["name"])
        assert np.array_equal(t["dw"][i], rec["dw"][i]), ("dw", c["name"])
        assert np.array_equal(m.get_weight(i), newW[i]), ("w", c["name"])


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


def test_resnet18_images_and_graph_replay(T):
    """uint8 images through the NHWC16 input quantiser, then the step captured as a hipGraph and
    replayed on new data: each replay equals the oracle step (quantiser included)."""
    import niti_oracle as O
    import niti_resnet_ref as RR
    from niti_amd.resnet import ResNet18
    hw, batch, classes = 32, 2, 10
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=77)
    rng = np.random.default_rng(77)
    m = ResNet18(batch, hw, classes)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    img = T.zeros((batch, 3, hw, hw), dtype=T.uint8, device="cuda")
    lab = T.zeros(batch, dtype=T.int32, device="cuda")
    m.train_step_images(img, lab)          # warm-up (allocator), then restore the weights
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    g = T.cuda.CUDAGraph()
    imgs = [rng.integers(0, 256, (batch, 3, hw, hw)).astype(np.uint8) for _ in range(3)]
    labs = [rng.integers(0, classes, batch).astype(np.int32) for _ in range(3)]
    img.copy_(T.from_numpy(imgs[0]))
    lab.copy_(T.from_numpy(labs[0]))
    with T.cuda.graph(g):
        m.train_step_images(img, lab)      # capture only: nothing runs
    for step in range(2):
        img.copy_(T.from_numpy(imgs[step]))
        lab.copy_(T.from_numpy(labs[step]))
        g.replay()
        T.cuda.synchronize()
        x, a = O.quantize_images(imgs[step])
        W, _ = RR.train_step(convs, W, S, x, a, labs[step], classes=classes)
        for i in range(len(convs)):
            assert np.array_equal(m.get_weight(i), W[i]), (step, convs[i]["name"])


@pytest.mark.parametrize("world", [2, 3])
def test_resnet18_data_parallel_equals_full_batch(T, world):
    """Exact data parallelism (niti_amd.dp): `world` ranks of 2 images each, run as
    threads on one device through ThreadComm, equal one device stepping the whole batch bit for
    bit -- every rank's updated weights and logits, over two steps from uint8 images (the input
    quantiser's statistics are global too)."""
    import threading
    import niti_resnet_ref as RR
    from niti_amd.dp import ThreadComm
    from niti_amd.resnet import ResNet18
    hw, per, classes = 32, 2, 10
    convs = RR.resnet18_convs(hw, classes)
    W, S = RR.init_weights(convs, seed=5 + world)
    rng = np.random.default_rng(world)
    full = ResNet18(per * world, hw, classes)
    full.record = True
    comm = ThreadComm(world)
    ranks = [ResNet18(per, hw, classes, comm=comm.rank(r)) for r in range(world)]
    for m in [full] + ranks:
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
        m.record = True
    for step in range(2):
        img = rng.integers(0, 256, (per * world, 3, hw, hw)).astype(np.uint8)
        lab = rng.integers(0, classes, per * world).astype(np.int32)
        full.train_step_images(T.from_numpy(img).cuda(), T.from_numpy(lab).cuda())
        errs = []

        def run(r):
            try:
                sl = slice(r * per, (r + 1) * per)
                ranks[r].train_step_images(T.from_numpy(np.ascontiguousarray(img[sl])).cuda(),
                                           T.from_numpy(np.ascontiguousarray(lab[sl])).cuda())
            except Exception as e:  # noqa: BLE001
                errs.append(e)
                comm._bar.abort()

        th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        T.cuda.synchronize()
        ft = full.taps()
        for r, m in enumerate(ranks):
            t = m.taps()
            assert t["exp_logits"] == ft["exp_logits"], (step, r)
            assert np.array_equal(t["logits"], ft["logits"][r * per:(r + 1) * per]), (step, r)
            for i, c in enumerate(convs):
                assert np.array_equal(t["dw"][i], ft["dw"][i]), ("dw", step, r, c["name"])
                assert np.array_equal(m.get_weight(i), full.get_weight(i)), ("w", step, r, c["name"])


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
