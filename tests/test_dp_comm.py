"""niti_amd.dp collectives on the CPU: TorchComm over a world-2 gloo group (the RCCL path's
semantics: MAX of the range words, SUM of int32 gradients and of the quantiser's u64 statistics)
and ThreadComm's in-process exchange."""
import os
import sys
import threading

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from niti_amd.dp import TorchComm
    c = TorchComm()
    rng = torch.Generator().manual_seed(rank)
    r = torch.randint(0, 1 << 30, (64,), generator=rng, dtype=torch.int32)
    g = torch.randint(-1 << 20, 1 << 20, (300,), generator=rng, dtype=torch.int32)
    s = torch.tensor([rank * 1000 + 7, (1 << 40) + rank, 200 + rank, 255 - rank], dtype=torch.int64)
    r0, g0 = r.clone(), g.clone()
    c.all_max(r)
    c.all_sum(g)
    c.all_sum(s[:2])
    c.all_max(s[2:])
    torch.save((rank, r0, g0, r, g, s), out)
    dist.destroy_process_group()


def test_torch_comm_gloo_world2(tmp_path):
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    paths = [str(tmp_path / f"rank{r}.pt") for r in range(2)]
    ps = [ctx.Process(target=_worker, args=(r, 2, port, paths[r])) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    out = [torch.load(f, weights_only=True) for f in paths]
    (_, ra, ga, r1, g1, s1), (_, rb, gb, r2, g2, s2) = out
    assert torch.equal(r1, torch.maximum(ra, rb)) and torch.equal(r2, r1)
    assert torch.equal(g1, ga + gb) and torch.equal(g2, g1)
    assert s1.tolist() == [7 + 1007, (1 << 41) + 1, 201, 255] and torch.equal(s1, s2)


def test_thread_comm_cpu():
    from niti_amd.dp import ThreadComm
    world = 3
    comm = ThreadComm(world)
    ts = [torch.tensor([r, 10 - r, 5], dtype=torch.int32) for r in range(world)]
    us = [torch.tensor([r, -r], dtype=torch.int32) for r in range(world)]

    def run(r):
        c = comm.rank(r)
        c.all_max(ts[r])
        c.all_sum(us[r])

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for r in range(world):
        assert ts[r].tolist() == [2, 10, 5] and us[r].tolist() == [3, -3]
    with pytest.raises(ValueError):
        comm.rank(world)


def test_thread_comm_mismatch_fails_fast():
    """A shape mismatch raised by rank 0's reduction aborts the barrier: the peers fail at once
    (BrokenBarrierError) instead of waiting out the timeout, and rank 0 surfaces the ValueError."""
    import time
    from niti_amd.dp import ThreadComm
    comm = ThreadComm(2, timeout=60.0)
    errs = {}

    def run(r):
        try:
            comm.rank(r).all_sum(torch.zeros(2 + r, dtype=torch.int32))
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    t0 = time.monotonic()
    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(30)
    assert time.monotonic() - t0 < 10
    assert isinstance(errs[0], ValueError) and isinstance(errs[1], threading.BrokenBarrierError)
