"""The product's RCCL data-parallel path (niti_model_attach_comm, one process per GPU, exact mode).

World 1, one GPU (runs on every GPU box): the model attaches a one-rank RCCL communicator, so
every collective call site of the step runs on the hardware -- the two communicators (ranges on
the step stream, the gradient buckets split off with ncclCommSplit on the comm stream), the
bucket events, the per-bucket range launches and the NITI_SGD join -- and the result must equal
the model without a communicator bit for bit.

World 2 (only where torch sees >= 2 devices; the in-process transport of tests/test_dp_local.py
covers the multi-rank protocol on one GPU): each rank steps its slice of the batch through the
C++ model with the RCCL communicators, overlap on and off; rank 0 also steps the whole batch on
its own device and every rank's weights and logits must equal that run bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _n_devices():
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def _arch(arch, seed):
    """(arch id, in_hw, classes, weights, wscales, images' hw) of a test network: VGG-11 / VGG-16 at
    32 px, ResNet-18 at 64 px (the stem, the stride-2 projections, the 16-px row-segment convs)."""
    import niti_amd
    import niti_model_ref as R
    import niti_resnet_ref as RR
    if arch == "resnet18":
        convs = RR.resnet18_convs(64, 10)
        W, S = RR.init_weights(convs, seed=seed)
        return niti_amd.ARCH_RESNET18, 64, 10, W, S, 64
    layers = R.vgg11_layers() if arch == "vgg11" else R.vgg16_layers(32)
    W, S = R.init_weights(layers, seed=seed)
    return (niti_amd.ARCH_VGG11 if arch == "vgg11" else niti_amd.ARCH_VGG16), (32 if arch == "vgg16" else 0), 0, W, S, 32


def _rank(rank, world, port, overlap, arch, q):
    sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(rank)
    from niti_amd.model import NitiModel
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a_id, in_hw, classes, W, S, hw = _arch(arch, 29)
        b = 4 if arch == "vgg11" else 2
        rng = np.random.default_rng(7)
        imgs = rng.integers(0, 256, (2, b * world, 3, hw, hw)).astype(np.uint8)
        labs = rng.integers(0, 10, (2, b * world)).astype(np.int32)
        uid = [NitiModel.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        m = NitiModel(a_id, b, in_hw, classes)
        m.attach_comm(uid[0], rank, world, exact=True)
        m.set_overlap(overlap)
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
        for step in range(2):
            sl = slice(rank * b, (rank + 1) * b)
            m.train_step_images(torch.from_numpy(imgs[step, sl].copy()).cuda(), torch.from_numpy(labs[step, sl].copy()).cuda())
        torch.cuda.synchronize()
        out = {"w": [m.get_weight(i) for i in range(len(W))], "logits": m.logits()}
        if rank == 0:
            full = NitiModel(a_id, b * world, in_hw, classes)
            for i, (w, s) in enumerate(zip(W, S)):
                full.set_weight(i, w, s)
            for step in range(2):
                full.train_step_images(torch.from_numpy(imgs[step]).cuda(), torch.from_numpy(labs[step]).cuda())
            torch.cuda.synchronize()
            out["full_w"] = [full.get_weight(i) for i in range(len(W))]
            out["full_logits"] = full.logits()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("arch,overlap", [("vgg11", False), ("vgg11", True), ("vgg16", False), ("resnet18", False)])
def test_rccl_world1_equals_no_comm(arch, overlap):
    """resnet18: the C++ ResNet driver's attach_comm (ncclCommSplit, the split agreement, the
    plan_buckets SUMs on the comm stream, every range MAX on the step stream) on hardware."""
    if _n_devices() < 1:
        pytest.skip("no GPU")
    import torch
    sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    from niti_amd.model import NitiModel
    a_id, in_hw, classes, W, S, hw = _arch(arch, 23)
    b = 8 if arch == "vgg11" else 4
    rng = np.random.default_rng(5)
    imgs = rng.integers(0, 256, (2, b, 3, hw, hw)).astype(np.uint8)
    labs = rng.integers(0, 10, (2, b)).astype(np.int32)
    runs = []
    for comm in (True, False):
        m = NitiModel(a_id, b, in_hw, classes)
        if comm:
            m.attach_comm(NitiModel.unique_id(), 0, 1, exact=True)
        m.set_overlap(overlap)
        for i, (w, s) in enumerate(zip(W, S)):
            m.set_weight(i, w, s)
        for step in range(2):
            m.train_step_images(torch.from_numpy(imgs[step]).cuda(), torch.from_numpy(labs[step]).cuda())
        torch.cuda.synchronize()
        runs.append(([m.get_weight(i) for i in range(len(W))], m.logits()))
        del m
    (wc, (lc, ec)), (wn, (ln, en)) = runs
    assert ec == en and np.array_equal(lc, ln)
    for i in range(len(W)):
        assert np.array_equal(wc[i], wn[i]), i


@pytest.mark.skipif(_n_devices() < 2, reason="needs >= 2 GPUs (one rank per GPU over RCCL)")
@pytest.mark.parametrize("arch,overlap", [("vgg11", True), ("vgg11", False), ("resnet18", False)])
def test_rccl_dp_matches_full_batch(arch, overlap):
    import torch.multiprocessing as mp
    world = 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, overlap, arch, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    full_w, (fl, fe) = res[0]["full_w"], res[0]["full_logits"]
    b = fl.shape[0] // world
    for r in range(world):
        lg, e = res[r]["logits"]
        assert e == fe and np.array_equal(lg, fl[r * b:(r + 1) * b]), r
        for i, w in enumerate(res[r]["w"]):
            assert np.array_equal(w, full_w[i]), (r, i)
