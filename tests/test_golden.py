"""Committed fixtures (tests/golden/niti_golden.npz, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces every fixture bit for bit (it pins the restatement against
drift; parity with the reference itself is unpinned).
GPU: the HIP path reproduces the same fixtures through the C ABI.
"""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "niti_golden.npz")
GEOMS = [(2, 8, 8, 16, 3, 1, 1), (3, 6, 9, 8, 3, 2, 1), (2, 5, 12, 12, 5, 1, 0)]  # as make_golden.py


@pytest.fixture(scope="module")
def G():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _onehot(labels, classes):
    oh = np.zeros((len(labels), classes), np.int32)
    oh[np.arange(len(labels)), labels] = 1
    return oh


# ------------------------------------------------------------------------------ CPU (oracle)
def test_golden_scalar_rules(oracle, G):
    for i, s in enumerate(G["psto_shifts"]):
        assert np.array_equal(oracle.psto(G["psto_vals"], int(s)), G["psto_out"][i]), int(s)
    off = 0
    for n, want in zip(G["range_lens"], G["range_cases"]):
        assert oracle.range_estimate(G["range_vals"][off:off + n]) == want
        off += n


@pytest.mark.parametrize("gi", range(len(GEOMS)))
def test_golden_conv_oracle(oracle, G, gi):
    n, ci, h, co, k, s, p = GEOMS[gi]
    g = oracle.geom(n, ci, h, h, co, k, stride=s, pad=p)
    x, w, dy = G[f"g{gi}_x"], G[f"g{gi}_w"], G[f"g{gi}_dy"]
    y, e, _, _ = oracle.conv_fwd(g, x, w, -7, int(G[f"g{gi}_wscale"]))
    assert np.array_equal(y, G[f"g{gi}_y"]) and e == G[f"g{gi}_exp"]
    dw, bw, _, _ = oracle.conv_wgrad(g, x, dy)
    assert np.array_equal(dw, G[f"g{gi}_dw"]) and bw == G[f"g{gi}_bw"]
    dx, inc, _, _ = oracle.conv_dgrad(g, dy, w)
    assert np.array_equal(dx, G[f"g{gi}_dx"]) and inc == G[f"g{gi}_dinc"]


def test_golden_small_ops_oracle(oracle, G):
    dwT, bw, _, _ = oracle.matmul(G["mm_B"], G["mm_A"])
    assert np.array_equal(dwT, G["mm_dwT"]) and bw == G["mm_bw"]
    x = G["pool_x"]
    assert np.array_equal(oracle.maxpool(x), G["pool_y"])
    assert np.array_equal(oracle.maxpool_grad(x, G["pool_y"], G["pool_dy"]), G["pool_dx"])
    assert np.array_equal(oracle.relu(x), G["relu_y"])
    assert np.array_equal(oracle.relu_grad(x, oracle.relu(x)), G["relu_dx"])
    lg = oracle.loss_grad(G["loss_logits"], int(G["loss_ascale"]), _onehot(G["loss_labels"], 12))
    assert np.array_equal(lg, G["loss_grad"])


def _lenet_weights(G):
    W = [G[f"lenet_w{i}"] for i in range(4)]
    S = [int(G[f"lenet_s{i}"]) for i in range(4)]
    newW = [(W[i].astype(np.int16) + G[f"lenet_delta{i}"]).astype(np.int8) for i in range(4)]
    return W, S, newW


def test_golden_lenet_step_oracle(G):
    import niti_model_ref as R
    W, S, newW = _lenet_weights(G)
    got, rec = R.train_step(R.lenet_layers(), W, S, G["lenet_x"], int(G["lenet_exp_in"]), G["lenet_labels"])
    assert np.array_equal(rec["logits"], G["lenet_logits"]) and rec["exp"][-1] == G["lenet_exp_out"]
    for i in range(4):
        assert np.array_equal(got[i], newW[i]), i


# ------------------------------------------------------------------------------ GPU (HIP path)
@pytest.fixture(scope="module")
def T():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import niti_amd  # noqa: F401  (fails loudly without the HIP library)
    return torch


def _dev(T, a):
    return T.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("gi", range(len(GEOMS)))
def test_golden_conv_hip(T, G, gi):
    from niti_amd import ops
    n, ci, h, co, k, s, p = GEOMS[gi]
    gg = ops.geom(n, ci, h, h, co, k, stride=s, pad=p)
    x16 = ops.nchw_to_nhwc16(_dev(T, G[f"g{gi}_x"]))
    w16 = ops.oihw_to_ohwi16(_dev(T, G[f"g{gi}_w"]))
    dy16 = ops.nchw_to_nhwc16(_dev(T, G[f"g{gi}_dy"]))
    amax = ops.new_range()
    e = T.zeros(1, dtype=T.int8, device="cuda")
    y16 = ops.requant_act(ops.conv_fwd_acc(gg, x16, w16, amax), amax, exp_in=_dev(T, np.array([-7], np.int8)),
                          wscale=_dev(T, np.array([int(G[f"g{gi}_wscale"])], np.int8)), exp_out=e)
    oh = ow = (h + 2 * p - k) // s + 1
    y = y16.cpu().numpy()[:, :co].reshape(n, oh, ow, co).transpose(0, 3, 1, 2)
    assert np.array_equal(y, G[f"g{gi}_y"]) and int(e.item()) == int(G[f"g{gi}_exp"])
    amax = ops.new_range()
    wacc = ops.conv_wgrad_acc(gg, x16, dy16)
    ops.absmax(wacc, amax)
    dw = ops.requant_grad(wacc, amax, rule=2).cpu().numpy()[..., :ci].transpose(0, 3, 1, 2)
    assert np.array_equal(dw, G[f"g{gi}_dw"])
    amax = ops.new_range()
    dacc = ops.conv_dgrad_acc(gg, dy16, ops.ohwi16_to_ihwo16(w16, ci), amax)
    dx = ops.requant_act(dacc, amax).cpu().numpy()[:, :ci].reshape(n, h, h, ci).transpose(0, 3, 1, 2)
    assert np.array_equal(dx, G[f"g{gi}_dx"])


@pytest.mark.gpu
def test_golden_lenet_step_hip(T, G):
    import niti_amd
    from niti_amd.model import NitiModel
    W, S, newW = _lenet_weights(G)
    m = NitiModel(niti_amd.ARCH_LENET, 4)
    for i in range(4):
        m.set_weight(i, W[i], S[i])
    m.train_step(_dev(T, G["lenet_x"]), int(G["lenet_exp_in"]), _dev(T, G["lenet_labels"]))
    logits, e = m.logits()
    assert np.array_equal(logits, G["lenet_logits"]) and e == int(G["lenet_exp_out"])
    for i in range(4):
        assert np.array_equal(m.get_weight(i), newW[i]), i
