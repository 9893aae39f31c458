"""The reference's snapshot format (Variable::save / Variable::load, express/Expr.cpp:833-965).

CPU: the hand-written flatbuffer encoder / decoder round-trips int8 parameters as TrainableParam
Blob ops with the reference's default names; the decoder reads the reference's own MNN model files
(benchmark/models/*.mnn, when /root/reference is present) into self-consistent nets; malformed
files are ValueError.  GPU: a model restored from a .mnn snapshot continues training exactly like
the model that wrote it."""
import os

import numpy as np
import pytest

from niti_amd import mnn_snapshot as M

REF_MODELS = "/root/reference/execution-engine/benchmark/models"


def test_encode_decode_round_trip(tmp_path):
    rng = np.random.default_rng(4)
    W = [rng.integers(-128, 128, s).astype(np.int8) for s in [(20, 1, 5, 5), (52, 20, 5, 5), (10, 500, 1, 1)]]
    net = M.decode_net(M.encode_params(W))
    assert net["tensorName"] == ["TrainableParam1", "TrainableParam2", "TrainableParam3"]
    for i, (op, w) in enumerate(zip(net["ops"], W)):
        assert op["name"] == f"TrainableParam{i + 1}" and op["type"] == M.OP_TRAINABLE_PARAM
        assert op["main_type"] == M.OP_PARAM_BLOB and op["outputIndexes"].tolist() == [i]
        assert op["inputIndexes"].tolist() == []
        b = op["blob"]
        assert b["dims"] == list(w.shape) and b["dataType"] == M.DT_INT8 and b["dataFormat"] == M.FMT_NCHW
        assert np.array_equal(b["data"].reshape(w.shape), w)
    p = str(tmp_path / "s.mnn")
    M.save(p, W, [-7, -8, -9], meta={"arch": 1})
    W2, S2, meta = M.load(p)
    assert S2 == [-7, -8, -9] and meta["arch"] == 1
    assert all(np.array_equal(a, b) for a, b in zip(W, W2))
    os.remove(p + ".wscale.json")
    W3, S3, _ = M.load(p)  # no side-car: the weights alone, as Variable::load returns them
    assert S3 is None and all(np.array_equal(a, b) for a, b in zip(W, W3))


def test_load_rejects_malformed(tmp_path):
    p = str(tmp_path / "bad.mnn")
    for blob in (b"", b"\x00" * 3, b"\xff" * 64, M.encode_params([np.zeros((2, 2, 1, 1), np.int8)])[:-12]):
        open(p, "wb").write(blob)
        with pytest.raises(ValueError):
            M.load(p)
    open(p, "wb").write(M.encode_params([np.zeros((2, 2, 1, 1), np.int8)]))
    open(p + ".wscale.json", "w").write('{"wscale": [1, 2]}')
    with pytest.raises(ValueError):
        M.load(p)  # 1 parameter, 2 scales
    open(p + ".wscale.json", "w").write('{"wscale": "x"}')
    with pytest.raises(ValueError):
        M.load(p)


@pytest.mark.parametrize("name,first_ops", [("squeezenetv1.1.mnn", ["data", "conv1"]),
                                            ("mobilenet-v1-1.0.mnn", ["input", "MobilenetV1/MobilenetV1/Conv2d_0/Conv2D"])])
def test_decode_reference_model_files(name, first_ops):
    """The decoder on flatbuffers the reference's MNN converter wrote: op names, every output index
    inside tensorName, the first op an Input (OpType 34)."""
    path = os.path.join(REF_MODELS, name)
    if not os.path.exists(path):
        pytest.skip("reference tree not present")
    net = M.decode_net(open(path, "rb").read())
    assert [op["name"] for op in net["ops"][:2]] == first_ops
    assert net["ops"][0]["type"] == 34
    n = len(net["tensorName"])
    assert n > 0 and all(op["outputIndexes"] is not None and (op["outputIndexes"] < n).all() for op in net["ops"])


@pytest.mark.gpu
def test_model_resume_from_mnn_snapshot(tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import niti_amd
    import niti_model_ref as R
    from niti_amd.model import NitiModel
    rng = np.random.default_rng(12)
    layers = R.lenet_layers()
    W, S = R.init_weights(layers, seed=12)
    batch = 16
    xs = [rng.integers(-127, 128, (batch, 1, 28, 28)).astype(np.int8) for _ in range(2)]
    ls = [rng.integers(0, 10, batch).astype(np.int32) for _ in range(2)]
    dev = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    m = NitiModel(niti_amd.ARCH_LENET, batch)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    m.train_step(dev(xs[0]), -3, dev(ls[0]))
    p = str(tmp_path / "mnist.snapshot.mnn")
    m.save_mnn(p)
    W1, S1, _ = M.load(p)
    W1_ref, _ = R.train_step(layers, W, S, xs[0], -3, ls[0])
    assert all(np.array_equal(a, b) for a, b in zip(W1, W1_ref)) and S1 == list(S)
    m2 = NitiModel(niti_amd.ARCH_LENET, batch)
    with pytest.raises(ValueError):
        os.rename(p + ".wscale.json", p + ".side")
        m2.load_mnn(p)  # fresh model: no scales of its own and no side-car
    os.rename(p + ".side", p + ".wscale.json")
    m2.load_mnn(p)
    m.train_step(dev(xs[1]), -3, dev(ls[1]))
    m2.train_step(dev(xs[1]), -3, dev(ls[1]))
    W2_ref, _ = R.train_step(layers, W1_ref, S, xs[1], -3, ls[1])
    for i in range(len(layers)):
        assert np.array_equal(m.get_weight(i), W2_ref[i]) and np.array_equal(m2.get_weight(i), W2_ref[i])
