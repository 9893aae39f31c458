"""Data-parallel exact mode on CPU: world_size 2 over gloo (127.0.0.1).

The device path (niti_model_attach_comm) shards the batch and keeps every rank bit-identical to
one device running the whole batch with two collectives per layer: all-reduce(MAX) of every
range estimate before its requantisation, and all-reduce(SUM) of the int32 weight gradient
before its range estimate.  This test runs exactly that protocol with the
oracle's arithmetic on two CPU ranks and checks the sharded results against the single-process
full batch, plus the control plane bench.py uses (NCCL unique-id broadcast, max of rank times).
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

WORLD = 2
GEO = (4, 6, 8, 10, 3, 1, 1)  # n, ci, h, co, k, stride, pad


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _requant_fwd_with(acc, m, O):
    """NITI_Conv_Int8.cpp:255-307 with the range taken from a (global) max m."""
    bw = O.range_estimate(np.array([m], np.int32))
    shift = bw - 7
    if shift > 1:
        return O.psto(acc, shift)
    if shift == 1:
        return O.psto(acc, 2)
    return acc.astype(np.int8).astype(np.int32)


def _requant_wgrad_with(acc, m, O):
    """NITI_GradientConv_Int8.cpp:272-296 with the range of the all-reduced gradient."""
    bw = O.range_estimate(np.array([m], np.int32))
    if bw == 0:
        return np.zeros_like(acc)
    return O.psto(acc, bw - 2)


def _data():
    import niti_oracle as O
    n, ci, h, co, k, s, p = GEO
    rng = np.random.default_rng(77)
    x = O.synth_x(rng, (n, ci, h, h))
    w, ws = O.synth_w(rng, (co, ci, k, k))
    g = O.geom(n, ci, h, h, co, k, stride=s, pad=p)
    dy = O.synth_dy(rng, (n, co, g.oh, g.ow))
    return x, w, ws, dy


def _rank(rank, port, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import niti_oracle as O
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=WORLD)
    try:
        n, ci, h, co, k, s, p = GEO
        x, w, _, dy = _data()
        sh = n // WORLD
        xs, dys = x[rank * sh:(rank + 1) * sh], dy[rank * sh:(rank + 1) * sh]
        g = O.geom(sh, ci, h, h, co, k, stride=s, pad=p)
        # forward: local accumulators, global range by MAX
        acc, _ = O.conv_fwd_acc(g, xs, w)
        m = torch.tensor([int(np.abs(acc.astype(np.int64)).max())], dtype=torch.int64)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        y = _requant_fwd_with(acc, int(m.item()), O)
        # weight gradient: local int32 partial sums, SUM, then the range of the sum
        wacc, _ = O.conv_wgrad_acc(g, xs, dys)
        t = torch.from_numpy(wacc.astype(np.int64))
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        tot = t.numpy().astype(np.int32)
        dw = _requant_wgrad_with(tot, int(np.abs(tot.astype(np.int64)).max()), O)
        # control plane of bench.py: unique-id broadcast and max of the rank timings
        uid = [b"\x01" * 128 if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        tm = torch.tensor([0.5 + rank], dtype=torch.float64)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        out_q.put((rank, y, dw, uid[0], float(tm.item())))
    finally:
        dist.destroy_process_group()


def test_dp_exact_mode_matches_full_batch(oracle):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(WORLD)]
    for pr in procs:
        pr.start()
    res = {}
    for _ in range(WORLD):
        r, y, dw, uid, tm = q.get(timeout=120)
        res[r] = (y, dw, uid, tm)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    n, ci, h, co, k, s, p = GEO
    x, w, ws, dy = _data()
    g = oracle.geom(n, ci, h, h, co, k, stride=s, pad=p)
    y_full, _, _, _ = oracle.conv_fwd(g, x, w, -7, ws)
    dw_full, _, _, _ = oracle.conv_wgrad(g, x, dy)
    sh = n // WORLD
    for r in range(WORLD):
        y, dw, uid, tm = res[r]
        assert np.array_equal(y.astype(np.int8), y_full[r * sh:(r + 1) * sh]), r
        assert np.array_equal(dw.astype(np.int8), dw_full), r
        assert uid == b"\x01" * 128 and tm == 0.5 + (WORLD - 1)


def test_dp_shard_local_ranges_are_not_exact(oracle):
    """Why exact mode needs the MAX all-reduce: shard-local ranges generally requantise the
    same accumulators differently from the full batch (so 'fast mode' is labelled non-parity)."""
    n, ci, h, co, k, s, p = GEO
    x, w, ws, _ = _data()
    x = x.copy()
    x[0] = 127  # a large first image: shard 0's range differs from shard 1's
    g = oracle.geom(n, ci, h, h, co, k, stride=s, pad=p)
    y_full, _, acc_full, _ = oracle.conv_fwd(g, x, w, -7, ws)
    sh = n // WORLD
    g1 = oracle.geom(sh, ci, h, h, co, k, stride=s, pad=p)
    y1, _, _, _ = oracle.conv_fwd(g1, x[sh:], w, -7, ws)
    assert not np.array_equal(y1, y_full[sh:])
