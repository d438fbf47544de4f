"""RCCL bootstraps of the native cascade.

``DeviceGroup``  P thread-ranks over GPUs 0..P-1 of THIS process: one ``ncclCommInitAll``, one
                 communicator + device context per GPU, kept between fits (buffers stay warm).
                 ``transport="loopback"`` runs the same ranks on fewer GPUs with host-staged
                 exchanges (rehearsals on one GPU).  Creating an RCCL group runs the preflight
                 (every op of the cascade driver with checked payloads, csrc/cascade/exercise.cpp).
``RcclRank``     one rank per process (torchrun): rank 0 draws the ncclUniqueId, the launcher's
                 store (``torch.distributed``, any backend, e.g. gloo) distributes it, every process
                 calls ``ncclCommInitRank`` on its own GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import _native as N


def rccl_info() -> dict:
    """RCCL the device library was built against and the one it runs on, with the library path: the
    librccl of those headers, loaded explicitly (csrc/hip/rccl_api.h), not the copy PyTorch bundles."""
    h, r = ctypes.c_int32(0), ctypes.c_int32(0)
    path = ctypes.create_string_buffer(512)
    N.hip().svmd_rccl_info(ctypes.byref(h), ctypes.byref(r), path, 512)

    def ver(c):
        return f"{c // 10000}.{c // 100 % 100}.{c % 100}" if c else "unknown"

    return {"rccl_header": ver(h.value), "rccl_runtime": ver(r.value), "rccl_path": path.value.decode(),
            "rccl_skew": h.value != r.value}


class DeviceGroup:
    _shared: dict = {}

    def __init__(self, world: int, transport: str = "auto", comm_timeout_s: float = 600.0):
        self.world = world
        self.handle = N.hip().svmd_cascade_group_create(int(world), transport.encode(), float(comm_timeout_s))
        if not self.handle:
            raise N.NativeError(N.last_error())
        self.transport = transport

    @property
    def broken(self) -> bool:
        """True once a failed fit / exercise aborted the communicators (the group cannot be used)."""
        return bool(self.handle) and bool(N.hip().svmd_cascade_group_broken(self.handle))

    def exercise(self, script: str, timeout_s: float = 20.0) -> None:
        """Run a transport script (exercise.cpp syntax) with checked payloads on every rank."""
        rc = N.hip().svmd_cascade_group_exercise(self.handle, script.encode(), float(timeout_s))
        if rc != 0:
            raise N.NativeError(N.last_error())

    @classmethod
    def shared(cls, world: int, transport: str = "auto") -> "DeviceGroup":
        """A process-wide group per (world, transport): communicators are created once, and again
        after a failure aborted them."""
        g = cls._shared.get((world, transport))
        if g is not None and (not g.handle or g.broken):
            g.close()
            g = None
        if g is None:
            g = cls._shared[(world, transport)] = cls(world, transport)
        return g

    @classmethod
    def release_shared(cls) -> None:
        for g in cls._shared.values():
            g.close()
        cls._shared.clear()

    def close(self) -> None:
        if self.handle:
            N.hip().svmd_cascade_group_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RcclRank:
    def __init__(self, device: int, uid: bytes, world: int, rank: int, comm_timeout_s: float = 600.0):
        self.device, self.world, self.rank = device, world, rank
        buf = np.frombuffer(uid, dtype=np.uint8).copy()
        self.handle = N.hip().svmd_cascade_rank_create(int(device), N.ptr(buf), int(world), int(rank),
                                                      float(comm_timeout_s))
        if not self.handle:
            raise N.NativeError(N.last_error())

    @staticmethod
    def unique_id() -> bytes:
        lib = N.hip()
        n = int(lib.svmd_nccl_unique_id_bytes())
        buf = np.zeros(n, dtype=np.uint8)
        N.check(lib.svmd_nccl_unique_id(N.ptr(buf), n), "svmd_nccl_unique_id")
        return buf.tobytes()

    @classmethod
    def from_torch_dist(cls, device: int, comm_timeout_s: float = 600.0) -> "RcclRank":
        """Every rank of an initialised torch.distributed group calls this collectively."""
        import torch.distributed as dist

        obj = [None]
        if dist.get_rank() == 0:
            try:
                obj[0] = cls.unique_id()
            except Exception as e:  # noqa: BLE001 - every rank must learn it, not wait in the broadcast
                obj[0] = f"{type(e).__name__}: {e}"
        dist.broadcast_object_list(obj, src=0)
        if isinstance(obj[0], str):
            raise N.NativeError(f"RCCL unique id on rank 0 failed: {obj[0]}")
        return cls(device, obj[0], dist.get_world_size(), dist.get_rank(), comm_timeout_s)

    def barrier(self) -> None:
        N.check(N.hip().svmd_cascade_rank_barrier(self.handle), "svmd_cascade_rank_barrier")

    def exercise(self, script: str, timeout_s: float = 20.0) -> None:
        """Collective: run a transport script (exercise.cpp syntax) with checked payloads."""
        rc = N.hip().svmd_cascade_rank_exercise(self.handle, script.encode(), float(timeout_s))
        if rc != 0:
            raise N.NativeError(N.last_error())

    def close(self) -> None:
        if self.handle:
            N.hip().svmd_cascade_rank_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
