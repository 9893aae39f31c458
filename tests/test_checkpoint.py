"""Parameter snapshots (mnistTrain.cpp:375-376 Variable::save).

CPU: the safetensors format round-trips int8 OIHW weights and the wscale side-car and rejects
malformed files.  GPU: a model restored from a snapshot taken mid-training continues with the
same next step as the model that wrote it, and that step matches the oracle's NITI_SGD step."""
import numpy as np
import pytest

from niti_amd.checkpoint import load_params, save_params


def test_params_round_trip(tmp_path):
    rng = np.random.default_rng(3)
    W = [rng.integers(-127, 128, s).astype(np.int8) for s in [(20, 1, 5, 5), (52, 20, 5, 5), (500, 832, 1, 1)]]
    S = [-7, -9, -11]
    p = str(tmp_path / "p.safetensors")
    save_params(p, W, S, arch=1)
    W2, S2, a = load_params(p)
    assert a == 1 and S2 == S
    assert all(w.dtype == np.int8 and np.array_equal(w, w2) for w, w2 in zip(W, W2))


def test_params_rejects_bad_input(tmp_path):
    p = str(tmp_path / "p.safetensors")
    with pytest.raises(ValueError):
        save_params(p, [np.zeros((1, 1, 1, 1), np.int32)], [0], arch=0)
    with pytest.raises(ValueError):
        save_params(p, [np.zeros((1, 1, 1, 1), np.int8)], [300], arch=0)
    with pytest.raises(ValueError):
        save_params(p, [np.zeros((1, 1, 1, 1), np.int8)], [], arch=0)
    from safetensors.numpy import save_file
    save_file({"x": np.zeros(3, np.int8)}, p)
    with pytest.raises(ValueError):
        load_params(p)
    # right format tag, missing / non-numeric / non-positive layer count or arch
    w = {"layer0.weight": np.zeros((1, 1, 1, 1), np.int8), "layer0.wscale": np.zeros(1, np.int8)}
    for meta in ({"format": "niti-int8-params-v1", "arch": "1"},
                 {"format": "niti-int8-params-v1", "arch": "1", "num_layers": "two"},
                 {"format": "niti-int8-params-v1", "arch": "1", "num_layers": "0"},
                 {"format": "niti-int8-params-v1", "num_layers": "1"},
                 {"format": "niti-int8-params-v1", "arch": "x", "num_layers": "1"}):
        save_file(w, p, metadata=meta)
        with pytest.raises(ValueError):
            load_params(p)


@pytest.mark.gpu
def test_model_resume_matches_oracle(tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import niti_amd
    import niti_model_ref as R
    from niti_amd.model import NitiModel
    rng = np.random.default_rng(9)
    layers = R.lenet_layers()
    W, S = R.init_weights(layers, seed=9)
    batch = 16
    xs = [rng.integers(-127, 128, (batch, 1, 28, 28)).astype(np.int8) for _ in range(2)]
    ls = [rng.integers(0, 10, batch).astype(np.int32) for _ in range(2)]
    dev = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    m = NitiModel(niti_amd.ARCH_LENET, batch)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    m.train_step(dev(xs[0]), -3, dev(ls[0]))
    p = str(tmp_path / "ck.safetensors")
    m.save(p)
    W1, S1, _ = load_params(p)
    W1_ref, _ = R.train_step(layers, W, S, xs[0], -3, ls[0])
    assert all(np.array_equal(a, b) for a, b in zip(W1, W1_ref)) and S1 == list(S)
    m2 = NitiModel(niti_amd.ARCH_LENET, batch)
    m2.load(p)
    m.train_step(dev(xs[1]), -3, dev(ls[1]))
    m2.train_step(dev(xs[1]), -3, dev(ls[1]))
    W2_ref, _ = R.train_step(layers, W1_ref, S, xs[1], -3, ls[1])
    for i in range(len(layers)):
        assert np.array_equal(m.get_weight(i), W2_ref[i])
        assert np.array_equal(m2.get_weight(i), W2_ref[i])
