"""Rank transports of the one-vs-rest trainer (models/multiclass.py): the classes are dealt over
ranks and the per-class alphas / intercepts are all-reduced.  (The Cascade SVM has its own native
transports, csrc/cascade: RCCL from C++ and a host-staged loopback.)

``TorchDistTransport`` wraps a ``torch.distributed`` group (backend "nccl" = RCCL over xGMI on
MI355X, or gloo); ``ThreadTransport`` runs P ranks as threads of one process (the native solvers
release the GIL) — CPU tests and single-GPU rehearsals of any P without a process group.
"""
from __future__ import annotations

import threading
from abc import ABC, abstractmethod
from typing import List, Optional

import torch


class Transport(ABC):
    rank: int
    world: int
    device: torch.device

    @abstractmethod
    def allreduce_(self, t: torch.Tensor, op: str) -> torch.Tensor: ...  # op: "min" | "max" | "sum"

    @abstractmethod
    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor: ...

    @abstractmethod
    def barrier(self) -> None: ...


class TorchDistTransport(Transport):
    """torch.distributed process group (backend "nccl" = RCCL on ROCm, or "gloo")."""

    _OPS = {"min": "MIN", "max": "MAX", "sum": "SUM"}

    def __init__(self, device: torch.device, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)

    def allreduce_(self, t, op):
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, self._OPS[op]), group=self.group)
        return t

    def broadcast_(self, t, src=0):
        self.dist.broadcast(t, src, group=self.group)
        return t

    def barrier(self):
        if self.device.type == "cuda":
            self.dist.barrier(group=self.group, device_ids=[self.device.index])
        else:
            self.dist.barrier(group=self.group)


class _ThreadGroup:
    def __init__(self, world: int):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots: List[Optional[torch.Tensor]] = [None] * world


class ThreadTransport(Transport):
    """P ranks as threads of one process sharing a ``_ThreadGroup``."""

    def __init__(self, group: _ThreadGroup, rank: int, device: torch.device):
        self.g = group
        self.rank = rank
        self.world = group.world
        self.device = torch.device(device)

    @staticmethod
    def create_group(world: int) -> _ThreadGroup:
        return _ThreadGroup(world)

    def _exchange(self, t: Optional[torch.Tensor]) -> List[Optional[torch.Tensor]]:
        self.g.slots[self.rank] = None if t is None else t.detach().clone()
        self.g.barrier.wait()
        snap = list(self.g.slots)
        self.g.barrier.wait()
        return snap

    def allreduce_(self, t, op):
        vals = self._exchange(t)
        acc = vals[0].clone()
        for v in vals[1:]:
            acc = {"min": torch.minimum, "max": torch.maximum, "sum": torch.add}[op](acc, v)
        t.copy_(acc)
        return t

    def broadcast_(self, t, src=0):
        vals = self._exchange(t if self.rank == src else None)
        if self.rank != src:
            t.copy_(vals[src])
        return t

    def barrier(self):
        self.g.barrier.wait()


def run_threads(world: int, fn, device_for_rank=lambda r: torch.device("cpu")):
    """Run ``fn(transport)`` on ``world`` thread-ranks; returns the per-rank results in rank order.
    Exceptions on any rank abort the group (broken barrier) and are re-raised.  Per-thread device
    state (contexts, scratch Grams; ops/device.py) is thread-local and released with the thread."""
    group = ThreadTransport.create_group(world)
    results: list = [None] * world
    errors: list = [None] * world

    def body(r):
        try:
            results[r] = fn(ThreadTransport(group, r, device_for_rank(r)))
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errors[r] = e
            group.barrier.abort()

    threads = [threading.Thread(target=body, args=(r,), name=f"rank{r}") for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for e in errors:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errors:
        if e is not None:
            raise e
    return results
