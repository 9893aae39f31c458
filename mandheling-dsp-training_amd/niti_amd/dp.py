"""Data-parallel exchange for the host-driven networks (niti_amd.resnet), SURVEY.md §8(e).

Exact mode makes every rank bit-identical to one device running the global batch.  The step
needs two collectives, both on int32 device tensors in program order:
  all_max  the range words of every forward / input-gradient / residual / pool range estimate
           (NITI_RangeEstimate spans the whole batch: NITI_Conv_Int8.cpp:260,
           NITI_DeConv_Int8.cpp:294) between the accumulate and the requantisation
  all_sum  each layer's int32 weight gradient (linear in the batch) before its range and NITI_SGD,
           and the input quantiser's statistics (MnistUtils.cpp:85-91)

TorchComm runs them through torch.distributed (backend "nccl" is RCCL on ROCm: one process per
GPU); ThreadComm runs N ranks as threads of one process on one device (tests and rehearsal): each
collective is a host barrier, a device reduction enqueued by rank 0 on the shared stream, and a
second barrier, so stream order follows the barriers.  The VGG / LeNet driver in
csrc/niti_model.hip has the same protocol in C++ (niti_model_attach_comm).
"""
from __future__ import annotations

import threading

import torch


class TorchComm:
    """The collectives over a torch.distributed process group (RCCL for CUDA tensors)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def all_max(self, t: torch.Tensor):
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)

    def all_sum(self, t: torch.Tensor):
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)


class ThreadComm:
    """N ranks as threads sharing one device and its current stream; rank(r) is rank r's handle."""

    def __init__(self, world: int, timeout: float = 120.0):
        if world < 1:
            raise ValueError("world >= 1")
        self.world = world
        self._bar = threading.Barrier(world, timeout=timeout)
        self._slots = [None] * world

    def rank(self, r: int) -> "_RankComm":
        if not 0 <= r < self.world:
            raise ValueError(f"rank {r} outside [0, {self.world})")
        return _RankComm(self, r)

    def _reduce(self, r: int, t: torch.Tensor, op: str):
        self._slots[r] = t
        self._bar.wait()
        if r == 0:
            try:
                ts = self._slots
                if any(x.shape != ts[0].shape or x.dtype != ts[0].dtype for x in ts):
                    raise ValueError("ranks disagree on the collective's tensor")
                acc = ts[0].clone()
                for x in ts[1:]:
                    if op == "max":
                        torch.maximum(acc, x, out=acc)
                    else:
                        acc.add_(x)
                for x in ts:
                    x.copy_(acc)
            except BaseException:
                # release the peers at once (BrokenBarrierError) instead of after the timeout,
                # and surface the real error on this rank
                self._bar.abort()
                raise
        self._bar.wait()
        self._slots[r] = None


class _RankComm:
    def __init__(self, group: ThreadComm, r: int):
        self.group, self.rank, self.world = group, r, group.world

    def all_max(self, t: torch.Tensor):
        self.group._reduce(self.rank, t, "max")

    def all_sum(self, t: torch.Tensor):
        self.group._reduce(self.rank, t, "sum")
