"""One cascade rank per process on the CPU oracle backend over a ``torch.distributed`` group.

``HostCommRank`` hands the native driver (``svm_cascade_rank_fit_cpu``, csrc/cascade/hostcomm.cpp)
a table of C callbacks that run the exchanges as gloo collectives on the driver's host buffers.  It
is the CPU twin of ``RcclRank`` (one rank per process under torchrun, RCCL from C++): the same
``run_cascade``, launched the same way, so ``torchrun --nproc-per-node 2 bench.py --gpus 2 --device
cpu`` and the multi-process CPU tests exercise the per-process path the 8-GPU run takes.
"""
from __future__ import annotations

import ctypes
import datetime
from ctypes import CFUNCTYPE, POINTER, c_double, c_int, c_int32, c_int64, c_void_p

import numpy as np
import torch

from .. import _native as N

_BCAST = CFUNCTYPE(c_int, c_void_p, c_void_p, c_int64, c_int32)
_ALLGATHER = CFUNCTYPE(c_int, c_void_p, c_void_p, c_int64, c_void_p)
_ALLREDUCE = CFUNCTYPE(c_int, c_void_p, POINTER(c_double), c_int64, c_int32)
_GATHER = CFUNCTYPE(c_int, c_void_p, c_void_p, c_int64, c_void_p, c_int32)
_SEND = CFUNCTYPE(c_int, c_void_p, c_void_p, c_int64, c_int32)
_RECV = CFUNCTYPE(c_int, c_void_p, c_void_p, c_int64, c_int32)
_BARRIER = CFUNCTYPE(c_int, c_void_p)


class SvmHostComm(ctypes.Structure):
    _fields_ = [("ctx", c_void_p), ("rank", c_int32), ("world", c_int32), ("bcast", _BCAST),
                ("allgather", _ALLGATHER), ("allreduce_f64", _ALLREDUCE), ("gather", _GATHER), ("send", _SEND),
                ("recv", _RECV), ("barrier", _BARRIER)]


def _bytes(ptr, nbytes: int) -> torch.Tensor:
    """A uint8 tensor aliasing nbytes of host memory at ptr (no copy)."""
    a = np.ctypeslib.as_array(ctypes.cast(ptr, POINTER(ctypes.c_uint8)), shape=(int(nbytes),))
    return torch.from_numpy(a)


class HostCommRank:
    """This process's rank of an initialised ``torch.distributed`` group (gloo) as a cascade rank.

    Every exchange is issued asynchronously and waited on with the fit's ``comm_timeout_s`` (the
    native driver's WaitPolicy deadline): a peer that failed -- and stays alive -- or stopped
    responding makes this rank's wait fail within that deadline instead of the process group's own
    (much longer) timeout, the MPI_Abort contract of the reference (mpi_svm_main3.cpp:420-428)."""

    device = "cpu"

    def __init__(self, group=None, comm_timeout_s: float = 600.0):
        import torch.distributed as dist

        # The rank's own gloo group unless one is given (collective: every rank constructs its rank
        # together): a collective this rank abandons after a timeout stays pending on it, and must not be
        # matched against the launcher's own control collectives on the default group afterwards.
        if group is None:
            group = dist.new_group(backend="gloo")
        self.dist, self.group = dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.timeout_s = float(comm_timeout_s)
        self.error: BaseException | None = None  # first exception raised inside a callback

        def done(work):
            if not work.wait(timeout=datetime.timedelta(seconds=self.timeout_s)):
                raise TimeoutError(f"collective did not complete within {self.timeout_s} s")

        def guard(fn):
            def wrapped(*a):
                try:
                    fn(*a)
                    return 0
                except BaseException as e:  # noqa: BLE001 - reported as a transport error, kept for the caller
                    if self.error is None:
                        self.error = e
                    return 1
            return wrapped

        g = self.group

        def bcast(_ctx, buf, nbytes, root):
            done(dist.broadcast(_bytes(buf, nbytes), src=dist.get_global_rank(g, root) if g else root, group=g,
                                async_op=True))

        def allgather(_ctx, send, nbytes, recv):
            out = _bytes(recv, nbytes * self.world)
            done(dist.all_gather(list(out.split(int(nbytes))), _bytes(send, nbytes).clone(), group=g, async_op=True))

        def allreduce(_ctx, buf, n, op):
            t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(int(n),)))
            done(dist.all_reduce(t, op=dist.ReduceOp.MIN if op == 0 else dist.ReduceOp.MAX, group=g, async_op=True))

        def gather(_ctx, send, nbytes, recv, root):
            dst = dist.get_global_rank(g, root) if g else root
            parts = list(_bytes(recv, nbytes * self.world).split(int(nbytes))) if self.rank == root else None
            done(dist.gather(_bytes(send, nbytes).clone(), gather_list=parts, dst=dst, group=g, async_op=True))

        def send(_ctx, buf, nbytes, peer):
            done(dist.isend(_bytes(buf, nbytes), dst=dist.get_global_rank(g, peer) if g else peer, group=g))

        def recv(_ctx, buf, nbytes, peer):
            done(dist.irecv(_bytes(buf, nbytes), src=dist.get_global_rank(g, peer) if g else peer, group=g))

        def barrier(_ctx):
            done(dist.barrier(group=g, async_op=True))

        # The CFUNCTYPE objects must outlive every native call: they are attributes of self.
        self._cbs = (_BCAST(guard(bcast)), _ALLGATHER(guard(allgather)), _ALLREDUCE(guard(allreduce)),
                     _GATHER(guard(gather)), _SEND(guard(send)), _RECV(guard(recv)), _BARRIER(guard(barrier)))
        self.comm = SvmHostComm(None, self.rank, self.world, *self._cbs)

    def barrier(self) -> None:
        self.dist.barrier(group=self.group)

    def fit(self, cfg, X, y, ids, n_total: int):
        """run_cascade on this rank's partition; returns the native svm_cascade_out pointer."""
        self.error = None
        if getattr(cfg, "comm_timeout_s", 0) > 0:
            self.timeout_s = float(cfg.comm_timeout_s)
        X = np.ascontiguousarray(X, dtype=np.float64)
        y = np.ascontiguousarray(y, dtype=np.int32)
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        p = N.core().svm_cascade_rank_fit_cpu(ctypes.addressof(self.comm), N.ptr(X), N.ptr(y), N.ptr(ids), X.shape[0],
                                              X.shape[1], int(n_total), ctypes.byref(cfg))
        if not p and self.error is not None:
            raise N.NativeError(f"{N.last_error()} (collective error: {self.error!r})") from self.error
        return p

    def close(self) -> None:
        pass


class HostCommDeviceRank:
    """This process's GPU rank with its exchanges over a ``torch.distributed`` group instead of RCCL
    (``svmd_cascade_rank_create_hostcomm``): device buffers are staged through host memory around the
    gloo collectives.  RCCL refuses two ranks on one GPU, this does not, so ``torchrun
    --nproc-per-node P bench.py --gpus P --transport hostcomm`` runs the per-process path of the N-GPU
    run (distributed decomposition, cascades) with P processes on ONE GPU: the same native drivers as
    ``RcclRank``, only the transport differs.  Used wherever an ``RcclRank`` is (its ``handle`` takes
    the same ``svmd_cascade_rank_*`` entry points).  Collective: every rank constructs it together."""

    def __init__(self, device: int, group=None, comm_timeout_s: float = 600.0):
        self.host = HostCommRank(group, comm_timeout_s)  # owns the callbacks: must outlive the handle
        self.device, self.world, self.rank = int(device), self.host.world, self.host.rank
        self.handle = N.hip().svmd_cascade_rank_create_hostcomm(ctypes.addressof(self.host.comm), self.device,
                                                               float(comm_timeout_s))
        if not self.handle:
            err = N.last_error()
            raise N.NativeError(f"{err} (collective error: {self.host.error!r})" if self.host.error else err)

    @property
    def error(self):
        return self.host.error

    def barrier(self) -> None:
        N.check(N.hip().svmd_cascade_rank_barrier(self.handle), "svmd_cascade_rank_barrier")

    def exercise(self, script: str, timeout_s: float = 20.0) -> None:
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
