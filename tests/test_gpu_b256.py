"""Full-tensor parity of the benchmarked configuration: one VGG-11 NITI step at batch 256.

bench.py times VGG-11 at batch 256 with autotuned GEMM plans (the tap-sharing weight-gradient
kernel split over K, split-K forward / input-gradient GEMMs, recompute plans).  Here the same
configuration -- uint8 images through the device quantiser, autotuned plans, then once more with
every tap-sharing layer forced to 6 and 8 K splits -- takes one step, and EVERY tap is compared
bit for bit with the oracle's reference-structured restatement (MNN C4 layout, 16x4 GEMM unit,
the grad graph's transposes / LeftPoolGrad / rot180; oracle/niti_oracle.c) run on the host's
cores: quantised input and ascale, each layer's requantised forward output, output gradient dy,
int8 weight gradient, updated weights, logits and their exponent.

The reference accumulates in float32 (Int8FunctionsOpt.cpp:211-226), which equals the exact
integer sum only while sum |x w| < 2^24.  The test prints, per layer, how many weight-gradient
outputs (and forward / input-gradient outputs) exceed that guard and how many int32 sums / int8
values a float32 sequential accumulation changes at this batch, so "bit-exact" states its own domain: the device matches the
exact sum everywhere, and matches the float32 reference wherever the printed counts are zero.
"""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B = 256


@pytest.fixture(scope="module")
def T():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import niti_amd  # noqa: F401
    return torch


@pytest.fixture(scope="module")
def case():
    import niti_model_ref as R
    import niti_oracle as O
    layers = R.vgg11_layers()
    W, S = R.init_weights(layers, seed=256)
    rng = np.random.default_rng(256)
    img = rng.integers(0, 256, (B, 3, 32, 32)).astype(np.uint8)
    labels = rng.integers(0, 10, B).astype(np.int32)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    O.set_threads(threads)
    t0 = time.perf_counter()
    x, ascale = O.quantize_images(img)
    newW, rec = R.train_step(layers, W, S, x, ascale, labels, impl="mnn", threads=threads, wgrad_stats=True)
    print(f"\noracle (reference-structured, {threads} threads): {time.perf_counter() - t0:.1f} s")
    for st in rec["wstats"]:
        print("  layer {layer}: wgrad outputs {outputs}, sum|p| >= 2^24: {guard}, int32 overflow: {overflow}, "
              "float32 accumulation changes {f32_int32_diff} int32 sums / {f32_int8_diff} int8 gradients "
              "(bw {bw} vs {bw_f32})".format(**st))
    for st in rec["fstats"]:
        print("  layer {layer} forward: outputs {outputs}, sum|p| >= 2^24: {guard}, int32 overflow: {overflow}, "
              "float32 accumulation changes {f32_int8_diff} int8 outputs / {exp_diff} exponents".format(**st))
    for st in rec["dstats"]:
        print("  layer {layer} input gradient: outputs {outputs}, sum|p| >= 2^24: {guard}, int32 overflow: "
              "{overflow}, float32 accumulation changes {f32_int32_diff} int32 sums / {f32_int8_diff} int8 outputs / "
              "{exp_diff} exponents".format(**st))
    assert all(st["overflow"] == 0 for st in rec["wstats"] + rec["fstats"] + rec["dstats"])
    return dict(layers=layers, W=W, S=S, img=img, labels=labels, x=x, ascale=ascale, newW=newW, rec=rec)


def _step_and_compare(T, case, prepare, keep_grads=True, overlap=True):
    import niti_amd
    from niti_amd._lib import NitiError
    from niti_amd.model import NitiModel
    layers, rec = case["layers"], case["rec"]
    m = NitiModel(niti_amd.ARCH_VGG11, B)
    m.keep_grads(keep_grads)
    m.set_overlap(overlap)
    img = T.from_numpy(case["img"]).cuda()
    lab = T.from_numpy(case["labels"]).cuda()
    for i, (w, s) in enumerate(zip(case["W"], case["S"])):
        m.set_weight(i, w, s)
    m.train_step_images(img, lab)  # fills the buffers the autotuner times on
    prepare(m)
    plans = m.plans()
    for i, (w, s) in enumerate(zip(case["W"], case["S"])):
        m.set_weight(i, w, s)
    m.train_step_images(img, lab)
    x, a = m.input()
    assert a == case["ascale"] and np.array_equal(x, case["x"])
    logits, e = m.logits()
    assert e == rec["exp"][-1] and np.array_equal(logits, rec["logits"])
    for i in range(len(layers)):
        if keep_grads or not layers[i]["pool"]:
            assert np.array_equal(m.tap(i, 0), rec["r"][i]), ("fwd", i, plans[(i, 0)])
        else:  # the pooled layers' 2x2 route went to the input gradients as codes: no pre-pool output
            with pytest.raises(NitiError):
                m.tap(i, 0)
        assert np.array_equal(m.tap(i, 2), rec["dy"][i]), ("dy", i)
        if keep_grads:
            assert np.array_equal(m.tap(i, 1), rec["dw"][i]), ("dw", i, plans[(i, 2)])
        assert np.array_equal(m.get_weight(i), case["newW"][i]), ("w", i)
    return plans


def test_vgg11_b256_autotuned_step_full_parity(T, case):
    from niti_amd.model import NitiModel
    try:
        plans = _step_and_compare(T, case, lambda m: m.autotune())
    finally:
        NitiModel.reset_plans()
    print("\nautotuned plans {(layer, phase): (bm, bn, splits, strategy)}:", plans)


@pytest.mark.parametrize("head_chain", [0, 1])
def test_vgg11_b256_bench_config_parity(T, case, head_chain):
    """The step exactly as bench.py times it: one stream, autotuned plans and keep_grads(False) -- no
    int8 weight-gradient copies, and the pooled layers' 2x2 routes recorded as codes by the forward
    kernels (conv0's and the row kernels' epilogues) and read by the next input gradient instead of
    the pre-pool output, which is then never written (NITI_CPUPoolGrad_Int8.cpp:21-77: the first
    window element >= the pooled value takes the gradient); the head's forward, loss gradient,
    weight and input gradients in the one head-chain launch
    (niti_head.hip, off by default; both ways).  Logits, every output gradient, every unpooled forward
    tap and every new weight against the oracle."""
    from niti_amd import _lib as L
    from niti_amd.model import NitiModel
    n0 = L.lib().niti_diag_head_chain_launches()
    L.lib().niti_diag_head_chain(head_chain)
    try:
        _step_and_compare(T, case, lambda m: m.autotune(), keep_grads=False, overlap=False)
    finally:
        L.lib().niti_diag_head_chain(0)
        NitiModel.reset_plans()
    ran = L.lib().niti_diag_head_chain_launches() - n0
    assert (ran > 0) == bool(head_chain)


@pytest.mark.parametrize("splits", [6, 8])
def test_vgg11_b256_taps_split_step_full_parity(T, case, splits):
    from niti_amd import ops
    from niti_amd.model import NitiModel

    def force(m):
        for i, l in enumerate(m.layers):
            g = ops.geom(B, l["c_in"], l["h"], l["w"], l["c_out"], l["kh"], pad=l["pad"])
            if ops.wgrad_taps_ok(g):
                m.set_plan(i, 2, (32, 32, splits, 2))

    try:
        plans = _step_and_compare(T, case, force)
    finally:
        NitiModel.reset_plans()
    assert plans[(3, 2)][:2] == (32, 32) and plans[(3, 2)][3] == 2


@pytest.mark.parametrize("splits", [1, 4])
def test_vgg11_b256_p16_split_step_full_parity(T, case, splits):
    """The P16 weight gradient (niti_wgrad.hip) forced on every layer it takes, unsplit and 4-way
    split-K (partials reduced by splitk_reduce_linear)."""
    from niti_amd.model import NitiModel

    def force(m):
        for i in range(len(m.layers)):
            if m.plan(i, 2)[:2] == (16, 16):
                m.set_plan(i, 2, (16, 16, splits, 2 if splits > 1 else 0))

    try:
        plans = _step_and_compare(T, case, force)
    finally:
        NitiModel.reset_plans()
    assert plans[(3, 2)] == (16, 16, splits, 2 if splits > 1 else 0)
