"""NITIInt8Train's input quantiser (execution-engine/tools/train/source/demo/MnistUtils.cpp:83-93).

CPU: the oracle's exact-statistics contract (niti_ref_image_quantize) against a hand-derived
known answer; against the float restatement of the reference expression (niti_ref_quantize_input_lanes),
which it equals wherever the float sums are exact; and the documented number of codes the float
readings (sequential, 4 / 8 / 16 lanes) change at the BASELINE input shapes.
GPU: the device quantiser (niti_image_stats / niti_image_quantize, and inside the model step)
bit-exact against the oracle, including statistics all-reduced over two half batches.
"""
import numpy as np
import pytest

import niti_oracle as O


def test_quant_known_answer():
    # an MNIST-shaped image of pixels {0, 255}: mean 127.5, std 127.5 (the literal divisor
    # batchSize * 28 * 28 is the pixel count), Y = -1 / +1, range 1 -> x = -127 / 127,
    # ascale = ceil(ln 1) - 7
    img = (np.indices((1, 1, 28, 28)).sum(0) % 2 * 255).astype(np.uint8)
    x, a = O.quantize_images(img)
    assert a == -7
    assert np.array_equal(x, np.where(img > 0, 127, -127).astype(np.int8))
    # not MNIST-shaped: MnistUtils.cpp:86 still divides the squared deviations by batchSize * 28 * 28,
    # so for a 2x2 image std = sqrt(4 * 127.5^2 / 784) = 127.5 / 14, range = 14, ascale = ceil(ln 14) - 7
    img = np.array([[[[0, 255], [255, 0]]]], np.uint8)
    x, a = O.quantize_images(img)
    assert a == -4
    assert x.tolist() == [[[[-127, 127], [127, -127]]]]
    st = O.image_stats(img)
    assert st.tolist() == [510, 2 * 255 * 255, 255, 255]


def test_quant_constant_batch_is_zero():
    # std == 0 is 0/0 in the reference; the contract quantises to zeros with ascale -7
    x, a = O.quantize_images(np.full((2, 1, 3, 3), 9, np.uint8))
    assert a == -7 and not x.any()


@pytest.mark.parametrize("shape", [(64, 1, 28, 28), (20, 1, 28, 28), (16, 3, 32, 32), (2, 3, 7, 5)])
def test_quant_matches_float_sequential_small(shape):
    """While every float partial sum is exact (S1 < 2^24 and few variance terms) the sequential float
    reading of MnistUtils.cpp:83-93 and the exact-statistics contract give the same codes."""
    rng = np.random.default_rng(sum(shape))
    img = rng.integers(0, 256, shape).astype(np.uint8)
    x, a = O.quantize_images(img)
    xf, af = O.quantize_input(img.astype(np.float32))
    assert a == af and np.array_equal(x, xf)
    assert x.min() >= -127 and x.max() <= 127


# The documented contract (DESIGN.md "Input quantiser", profiles/r04_quant_parity.txt): the device
# computes MnistUtils.cpp:83-93 over exact integer statistics; the reference sums in float in an
# order -ffast-math leaves to the compiler.  Per seed, BASELINE input shape and float order (lanes
# = interleaved partial sums, 1 = the C loop's sequential order): (differing int8 inputs, pixel
# values of 256 whose code differs).  Seeded uniform uint8 images, as tools/quant_parity.py.
QUANT_FLIPS = {
    (1, (256, 3, 32, 32)): {1: (0, 0), 4: (0, 0), 8: (0, 0), 16: (0, 0)},
    (5, (256, 3, 32, 32)): {1: (3018, 1), 4: (0, 0), 8: (0, 0), 16: (0, 0)},
    (1, (64, 1, 28, 28)): {1: (0, 0), 4: (0, 0), 8: (0, 0), 16: (0, 0)},
    (1, (64, 3, 224, 224)): {1: (0, 0), 4: (37728, 1), 8: (0, 0), 16: (0, 0)},
    (5, (64, 3, 224, 224)): {1: (37582, 1), 4: (0, 0), 8: (0, 0), 16: (0, 0)},
    (5, (128, 3, 224, 224)): {1: (300076, 4), 4: (0, 0), 8: (0, 0), 16: (74998, 1)},
}


@pytest.mark.parametrize("key", list(QUANT_FLIPS), ids=lambda k: f"seed{k[0]}-{'x'.join(map(str, k[1]))}")
def test_quant_contract_flip_counts(key):
    """Exact-statistics contract vs the float readings: the documented flip counts, each flip a
    whole pixel-value class moved by one code, the exponent (ascale) equal in every order."""
    seed, shape = key
    img = np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)
    x, a = O.quantize_images(img)
    f = img.astype(np.float32)
    for lanes, (flips, classes) in QUANT_FLIPS[key].items():
        xf, af = O.quantize_input(f, lanes)
        assert af == a, lanes
        d = x.astype(np.int16) - xf.astype(np.int16)
        assert np.abs(d).max() <= 1, lanes
        moved = np.unique(img[d != 0])
        assert (int((d != 0).sum()), int(moved.size)) == (flips, classes), lanes
        # the quantiser is a per-batch map of the 256 pixel values: a flip moves every pixel of a value
        assert int((d != 0).sum()) == int(np.isin(img, moved).sum()), lanes


def test_quant_split_statistics():
    """Data-parallel ranks: statistics summed / max-ed over shards give the global quantisation."""
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (8, 1, 28, 28)).astype(np.uint8)
    x, a = O.quantize_images(img)
    s0, s1 = O.image_stats(img[:4]), O.image_stats(img[4:])
    st = np.array([s0[0] + s1[0], s0[1] + s1[1], max(s0[2], s1[2]), max(s0[3], s1[3])], np.uint64)
    x0, a0 = O.quantize_images(img[:4], st, img.size)
    x1, a1 = O.quantize_images(img[4:], st, img.size)
    assert a0 == a1 == a
    assert np.array_equal(np.concatenate([x0, x1]), x)


@pytest.fixture(scope="module")
def T():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import niti_amd  # noqa: F401
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(64, 1, 28, 28), (5, 1, 28, 28), (256, 3, 32, 32), (3, 3, 7, 5), (1, 1, 1, 17)])
def test_quant_device_matches_oracle(T, shape):
    from niti_amd import ops
    rng = np.random.default_rng(shape[0] + shape[3])
    img = rng.integers(0, 256, shape).astype(np.uint8)
    d = T.from_numpy(img).cuda()
    st = ops.image_stats(d)
    assert st.cpu().numpy().astype(np.uint64).tolist() == O.image_stats(img).tolist()
    x, a = ops.image_quantize(d, st)
    xr, ar = O.quantize_images(img)
    assert int(a.item()) == ar
    assert np.array_equal(x.cpu().numpy(), xr)


@pytest.mark.gpu
def test_quant_device_constant_and_extremes(T):
    from niti_amd import ops
    for img in (np.full((2, 1, 4, 4), 200, np.uint8), np.array([[[[0, 255] * 8]]], np.uint8)):
        d = T.from_numpy(img).cuda()
        x, a = ops.image_quantize(d, ops.image_stats(d))
        xr, ar = O.quantize_images(img)
        assert int(a.item()) == ar and np.array_equal(x.cpu().numpy(), xr)


@pytest.mark.gpu
def test_quant_device_split_statistics(T):
    from niti_amd import ops
    rng = np.random.default_rng(8)
    img = rng.integers(0, 256, (6, 3, 32, 32)).astype(np.uint8)
    h0, h1 = T.from_numpy(img[:2].copy()).cuda(), T.from_numpy(img[2:].copy()).cuda()
    s0, s1 = ops.image_stats(h0), ops.image_stats(h1)
    st = T.stack([s0[0] + s1[0], s0[1] + s1[1], T.maximum(s0[2], s1[2]), T.maximum(s0[3], s1[3])])
    x0, a0 = ops.image_quantize(h0, st, img.size)
    x1, a1 = ops.image_quantize(h1, st, img.size)
    xr, ar = O.quantize_images(img)
    assert int(a0.item()) == int(a1.item()) == ar
    assert np.array_equal(np.concatenate([x0.cpu().numpy(), x1.cpu().numpy()]), xr)


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["lenet", "vgg11"])
def test_model_step_from_images_matches_oracle(T, arch):
    """The whole NITIInt8Train per-batch work from uint8 images: quantiser + NITI_SGD step."""
    import niti_amd
    import niti_model_ref as R
    from niti_amd.model import NitiModel
    layers = R.lenet_layers() if arch == "lenet" else R.vgg11_layers()
    a_id = niti_amd.ARCH_LENET if arch == "lenet" else niti_amd.ARCH_VGG11
    batch = 16 if arch == "lenet" else 6
    W, S = R.init_weights(layers, seed=31)
    m = NitiModel(a_id, batch)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    rng = np.random.default_rng(31)
    l0 = layers[0]
    for step in range(2):
        img = rng.integers(0, 256, (batch, l0["ci"], l0["h"], l0["h"])).astype(np.uint8)
        labels = rng.integers(0, 10, batch).astype(np.int32)
        x, ascale = O.quantize_images(img)
        newW, rec = R.train_step(layers, W, S, x, ascale, labels)
        m.train_step_images(T.from_numpy(img).cuda(), T.from_numpy(labels).cuda())
        xd, ad = m.input()
        assert ad == ascale and np.array_equal(xd, x), step
        logits, e = m.logits()
        assert e == rec["exp"][-1] and np.array_equal(logits, rec["logits"]), step
        for i in range(len(layers)):
            assert np.array_equal(m.get_weight(i), newW[i]), (step, i)
        W = newW
