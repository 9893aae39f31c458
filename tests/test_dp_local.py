"""The product's data-parallel protocol on one GPU.

`world` models of batch b, each driven by its own host thread on its own HIP stream and
attached to an in-process rank group (niti_model_attach_local): the step runs the exact calls,
order and streams of the RCCL path (two communicators: the quantiser statistics SUM/MAX and every
forward / input-gradient range MAX on the step stream; the int32 weight-gradient SUM of every
gradient bucket on the comm stream as soon as its weight gradients are in, followed there by the
bucket's ranges, joined by the step stream before NITI_SGD), with a transport that reduces on
the same device.  Exact mode must make every
rank bit-identical to ONE model stepping the concatenated batch of world * b images: same
weights, and each rank's activations / gradients equal its slice of the full batch's.
"""
import ctypes as C
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
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a rank thread hung"
    if errs:
        raise errs[0]


@pytest.mark.parametrize("arch,world,b,overlap,images", [
    ("vgg11", 2, 4, True, False),
    ("vgg11", 2, 4, False, False),
    ("vgg11", 2, 3, True, True),
    ("vgg11", 4, 2, True, True),
    ("lenet", 2, 8, True, True),
])
def test_local_dp_matches_full_batch(T, arch, world, b, overlap, images):
    import niti_amd
    import niti_model_ref as R
    from niti_amd.model import LocalGroup, NitiModel
    layers = R.lenet_layers() if arch == "lenet" else R.vgg11_layers()
    a_id = niti_amd.ARCH_LENET if arch == "lenet" else niti_amd.ARCH_VGG11
    W, S = R.init_weights(layers, seed=41)
    full = NitiModel(a_id, b * world)
    ranks = [NitiModel(a_id, b) for _ in range(world)]
    group = LocalGroup(world)
    for r, m in enumerate(ranks):
        m.attach_local(group, r, exact=True)
    for m in [full] + ranks:
        m.set_overlap(overlap)
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
    streams = [T.cuda.Stream() for _ in range(world)]
    rng = np.random.default_rng(41 + world)
    l0 = layers[0]
    for step in range(2):
        shape = (b * world, l0["ci"], l0["h"], l0["h"])
        labels = rng.integers(0, 10, b * world).astype(np.int32)
        ld = T.from_numpy(labels).cuda()
        if images:
            data = T.from_numpy(rng.integers(0, 256, shape).astype(np.uint8)).cuda()
            full.train_step_images(data, ld)
        else:
            data = T.from_numpy(rng.integers(-127, 128, shape).astype(np.int8)).cuda()
            full.train_step(data, -3, ld)
        T.cuda.synchronize()
        parts = [(data[r * b:(r + 1) * b].contiguous(), ld[r * b:(r + 1) * b].contiguous()) for r in range(world)]

        def rank_step(r):
            s = C.c_void_p(streams[r].cuda_stream)
            if images:
                ranks[r].train_step_images(parts[r][0], parts[r][1], stream=s)
            else:
                ranks[r].train_step(parts[r][0], -3, parts[r][1], stream=s)
            streams[r].synchronize()

        _in_threads([lambda r=r: rank_step(r) for r in range(world)])
        fl, fe = full.logits()
        for r, m in enumerate(ranks):
            sl = slice(r * b, (r + 1) * b)
            lg, e = m.logits()
            assert e == fe and np.array_equal(lg, fl[sl]), (step, r)
            if images:
                xf, af = full.input()
                xr, ar = m.input()
                assert ar == af and np.array_equal(xr, xf[sl]), (step, r)
            for i in range(len(layers)):
                assert np.array_equal(m.tap(i, 0), full.tap(i, 0)[sl]), ("fwd", step, r, i)
                assert np.array_equal(m.tap(i, 2), full.tap(i, 2)[sl]), ("dy", step, r, i)
                assert np.array_equal(m.tap(i, 1), full.tap(i, 1)), ("dw", step, r, i)
                assert np.array_equal(m.get_weight(i), full.get_weight(i)), ("w", step, r, i)


def test_local_dp_full_batch_is_oracle(T):
    """Anchor: the full-batch model of the cases above against the oracle's NITI_SGD step."""
    import niti_amd
    import niti_model_ref as R
    from niti_amd.model import LocalGroup, NitiModel
    import niti_oracle as O
    layers = R.vgg11_layers()
    W, S = R.init_weights(layers, seed=43)
    b, world = 3, 2
    ranks = [NitiModel(niti_amd.ARCH_VGG11, b) for _ in range(world)]
    group = LocalGroup(world)
    for r, m in enumerate(ranks):
        m.attach_local(group, r)
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
    rng = np.random.default_rng(43)
    img = rng.integers(0, 256, (b * world, 3, 32, 32)).astype(np.uint8)
    labels = rng.integers(0, 10, b * world).astype(np.int32)
    x, ascale = O.quantize_images(img)
    newW, rec = R.train_step(layers, W, S, x, ascale, labels)
    streams = [T.cuda.Stream() for _ in range(world)]

    def rank_step(r):
        ranks[r].train_step_images(T.from_numpy(img[r * b:(r + 1) * b].copy()).cuda(),
                                   T.from_numpy(labels[r * b:(r + 1) * b].copy()).cuda(),
                                   stream=C.c_void_p(streams[r].cuda_stream))
        streams[r].synchronize()

    _in_threads([lambda r=r: rank_step(r) for r in range(world)])
    for r, m in enumerate(ranks):
        lg, e = m.logits()
        assert e == rec["exp"][-1] and np.array_equal(lg, rec["logits"][r * b:(r + 1) * b])
        for i in range(len(layers)):
            assert np.array_equal(m.get_weight(i), newW[i]), (r, i)
