"""Transports for the Cascade SVM: the reference's MPI call sites re-expressed as
collectives over ``torch.distributed`` (RCCL over xGMI on MI355X, gloo on CPUs) or over threads.

| reference call site (mpi_svm_main*.cpp)            | Transport method                       |
|----------------------------------------------------|----------------------------------------|
| MPI_Bcast n_features / n_total (M3 :459-461)       | ``broadcast_int``                      |
| MPI_Bcast min/max (M3 :534-535)                    | ``allreduce_`` MIN / MAX of local stats |
| MPI_Bcast SV count + X/Y/alpha/ID (M3 :587-601)    | ``broadcast_int`` + ``broadcast_``     |
|                                                    |   of ONE packed (k, w+3) float64 buffer |
| tree MPI_Send/Recv count+4 arrays (M3 :689-716)    | ``send_rows`` / ``recv_rows``          |
| star MPI_Send/Recv to rank 0 (M2 :578-607,748-760) | ``gather_rows`` (counts all-gathered,  |
|                                                    |   max-padded ``dist.gather`` to rank 0) |
| MPI_Bcast converged flag (M3 :824, M2 :764)        | ``broadcast_int``                      |

Instead of four messages per SV set (X, Y, alpha, ID with tags 20-24), rows, labels, alphas and
IDs travel as one packed float64 buffer (IDs < 2^53 and +-1 labels are exact in float64), so each
exchange is a count plus one bulk transfer that stays on the device end to end.

``ThreadTransport`` runs P ranks as threads of one process (the native solvers release the GIL),
which gives CPU tests and single-GPU rehearsals of any P without a process group.
"""
from __future__ import annotations

import queue
import threading
from abc import ABC, abstractmethod
from typing import List, Optional

import torch


class Transport(ABC):
    rank: int
    world: int
    device: torch.device

    @abstractmethod
    def allreduce_(self, t: torch.Tensor, op: str) -> torch.Tensor: ...

    @abstractmethod
    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor: ...

    @abstractmethod
    def gather_rows(self, payload: torch.Tensor, dst: int = 0) -> Optional[List[torch.Tensor]]: ...

    @abstractmethod
    def send_rows(self, payload: torch.Tensor, dst: int) -> None: ...

    @abstractmethod
    def recv_rows(self, src: int, width: int) -> torch.Tensor: ...

    @abstractmethod
    def barrier(self) -> None: ...

    def broadcast_int(self, v: int, src: int = 0) -> int:
        t = torch.tensor([int(v)], dtype=torch.int64, device=self.device)
        self.broadcast_(t, src)
        return int(t.item())

    def broadcast_rows(self, payload: Optional[torch.Tensor], width: int, src: int = 0) -> torch.Tensor:
        """Count, then one bulk broadcast of a (k, width) float64 buffer from src."""
        k = self.broadcast_int(payload.shape[0] if self.rank == src else 0, src)
        if self.rank != src:
            payload = torch.empty((k, width), dtype=torch.float64, device=self.device)
        if k:
            self.broadcast_(payload, src)
        return payload


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

    def gather_rows(self, payload, dst=0):
        w = payload.shape[1]
        cnt = torch.tensor([payload.shape[0]], dtype=torch.int64, device=self.device)
        counts = torch.empty(self.world, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(counts, cnt, group=self.group)
        counts = counts.tolist()
        kmax = max(counts)
        if kmax == 0:
            return [torch.empty((0, w), dtype=torch.float64, device=self.device) for _ in range(self.world)] \
                if self.rank == dst else None
        padded = torch.zeros((kmax, w), dtype=torch.float64, device=self.device)
        padded[: payload.shape[0]] = payload
        bufs = [torch.empty_like(padded) for _ in range(self.world)] if self.rank == dst else None
        self.dist.gather(padded, bufs, dst=dst, group=self.group)
        if self.rank != dst:
            return None
        return [b[:c] for b, c in zip(bufs, counts)]

    def send_rows(self, payload, dst):
        cnt = torch.tensor([payload.shape[0]], dtype=torch.int64, device=self.device)
        self.dist.send(cnt, dst, group=self.group)
        if payload.shape[0]:
            self.dist.send(payload.contiguous(), dst, group=self.group)

    def recv_rows(self, src, width):
        cnt = torch.empty(1, dtype=torch.int64, device=self.device)
        self.dist.recv(cnt, src, group=self.group)
        k = int(cnt.item())
        out = torch.empty((k, width), dtype=torch.float64, device=self.device)
        if k:
            self.dist.recv(out, src, group=self.group)
        return out

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
        self.queues = {(s, d): queue.Queue() for s in range(world) for d in range(world)}


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

    def gather_rows(self, payload, dst=0):
        vals = self._exchange(payload)
        return [v.to(self.device) for v in vals] if self.rank == dst else None

    def send_rows(self, payload, dst):
        self.g.queues[(self.rank, dst)].put(payload.detach().clone())

    def recv_rows(self, src, width):
        out = self.g.queues[(src, self.rank)].get(timeout=3600)
        assert out.shape[1] == width
        return out.to(self.device)

    def barrier(self):
        self.g.barrier.wait()


def run_threads(world: int, fn, device_for_rank=lambda r: torch.device("cpu")):
    """Run ``fn(transport)`` on ``world`` thread-ranks; returns the per-rank results in rank order.
    Exceptions on any rank abort the group (broken barrier) and are re-raised."""
    group = ThreadTransport.create_group(world)
    results: list = [None] * world
    errors: list = [None] * world

    def body(r):
        try:
            results[r] = fn(ThreadTransport(group, r, device_for_rank(r)))
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errors[r] = e
            group.barrier.abort()

    threads = [threading.Thread(target=body, args=(r,), name=f"cascade-rank{r}") for r in range(world)]
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
