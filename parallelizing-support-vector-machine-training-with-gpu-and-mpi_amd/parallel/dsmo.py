"""Distributed SMO over the GPUs of one node (``--parallel smo``; csrc/hip/dsmo.hip).

ONE first-order SMO whose training points are split over P teams of workgroups -- one team per GPU
(P GPUs of this process, peer access between them) or, as a rehearsal, P teams on GPU 0 -- each with
its slab K(:, own) of the exact-integer RBF Gram.  The per-iteration arg-min / arg-max records cross
the GPUs over xGMI (uncached receive arrays, one fabric hop per iteration), and the second index's
kernel value K(i_high, i_low) is recomputed from the quantised rows, so every GPU applies the same
update: the result -- iterations, every alpha, b -- is the single-GPU trainer's, bit for bit.

The reference's multi-processor algorithm is the Cascade (mpi_svm_main2/3.cpp, ``CascadeSVM``); this
is the distributed-SMO design of its literature folder (papers/2006_Cao_SVM_MPI.pdf).
It needs integer pixel rows (the exact-integer Gram, e.g. MNIST); other data use the cascade.
"""
from __future__ import annotations

import ctypes
import time
from typing import Optional

import numpy as np

from .. import _native as N
from ..utils.config import SVMParams


def plan(n: int, world: int, ncu: int = 256, one_launch: bool = False) -> dict:
    """The team plan of a distributed solve (host only): threads per workgroup, points per thread,
    workgroups per team, records per sweep lane, points per workgroup and per team."""
    out = np.zeros(6, dtype=np.int64)
    rc = N.hip().svmd_dsmo_plan(int(n), int(world), int(ncu), int(one_launch), N.ptr(out))
    if rc != 0:
        raise N.NativeError(N.last_error())
    keys = ("threads", "points_per_thread", "workgroups_per_team", "records_per_lane", "slice", "team_width")
    return dict(zip(keys, (int(v) for v in out)))


class DsmoGroup:
    """Native distributed-SMO group: ``world`` teams on GPUs 0..world-1 (or all on GPU 0 with
    ``rehearsal=True``).  Buffers (rows, slabs, receive arrays) are kept between fits."""

    _shared: dict = {}

    def __init__(self, world: int, rehearsal: bool = False, timeout_s: float = 60.0):
        self.world, self.rehearsal = int(world), bool(rehearsal)
        self.handle = N.hip().svmd_dsmo_create(self.world, int(self.rehearsal), float(timeout_s))
        if not self.handle:
            raise N.NativeError(N.last_error())

    @classmethod
    def shared(cls, world: int, rehearsal: bool = False) -> "DsmoGroup":
        g = cls._shared.get((world, rehearsal))
        if g is None or not g.handle:
            g = cls._shared[(world, rehearsal)] = cls(world, rehearsal)
        return g

    @classmethod
    def release_shared(cls) -> None:
        for g in cls._shared.values():
            g.close()
        cls._shared.clear()

    def fit(self, X: np.ndarray, y: np.ndarray, params: Optional[SVMParams] = None, trace_cap: int = 0) -> dict:
        """Raw solve: alpha (host), result fields, phase times, team shape, column statistics."""
        from ..utils.data import check_labels, pixel_rows

        X = pixel_rows(X, "the distributed SMO (use CascadeSVM for other data)")
        n, d = X.shape
        y = check_labels(y, n)
        params = params or SVMParams()
        p = params.to_struct()
        alpha = np.empty(n, dtype=np.float64)
        r = N.SvmResult()
        tm = np.zeros(4, dtype=np.float64)
        shape = np.zeros(4, dtype=np.int32)
        mn = np.empty(d, dtype=np.float64)
        mx = np.empty(d, dtype=np.float64)
        trace = np.zeros((max(trace_cap, 0), 2), dtype=np.int64) if trace_cap > 0 else None
        rc = N.hip().svmd_dsmo_fit(self.handle, N.ptr(X), 1, N.ptr(y), n, d, ctypes.byref(p), N.ptr(alpha),
                                   ctypes.byref(r), N.ptr(tm), N.ptr(trace), max(trace_cap, 0), N.ptr(shape),
                                   N.ptr(mn), N.ptr(mx))
        if rc != 0:
            raise N.NativeError(N.last_error())
        out = {"alpha": alpha, "iterations": int(r.iterations), "b": float(r.b), "b_high": float(r.b_high),
               "b_low": float(r.b_low), "stop_reason": N.STOP_NAMES.get(int(r.stop_reason), str(r.stop_reason)),
               "n_sv": int(r.n_sv), "mn": mn, "mx": mx,
               "timings_ms": {"upload_minmax_ms": float(tm[0]), "quantise_slab_ms": float(tm[1]),
                              "smo_ms": float(tm[2]), "total_ms": float(tm[3])},
               "shape": {"threads": int(shape[0]), "points_per_thread": int(shape[1]),
                         "workgroups_per_team": int(shape[2]), "records_per_lane": int(shape[3])}}
        if trace is not None:
            out["trace"] = trace[: max(0, min(trace_cap, out["iterations"] - 1))]
        return out

    def close(self) -> None:
        if getattr(self, "handle", None):
            N.hip().svmd_dsmo_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DistributedSVC:
    """Estimator over a ``DsmoGroup`` (teams of this process) or a ``DsmoRank`` (this process's team
    of a per-process solve): ``fit`` / ``decision_function`` / ``predict`` / ``score``; the fitted
    model is an ``SVC`` (support vectors, dual coefficients, b, scaler) on this process's GPU."""

    def __init__(self, world: int = 1, rehearsal: bool = False, C: float = 10.0, gamma: float = 0.00125,
                 tol: float = 1e-5, eps: float = 1e-12, sv_tol: float = 1e-8, max_iter: int = 100000,
                 group: Optional[DsmoGroup] = None, rank: Optional["DsmoRank"] = None):
        self.params = SVMParams(C=C, gamma=gamma, tau=tol, eps=eps, sv_tol=sv_tol, max_iter=max_iter)
        self.world, self.rehearsal, self.group, self.rank = world, rehearsal, group, rank

    def fit(self, X: np.ndarray, y: np.ndarray, trace_cap: int = 0) -> "DistributedSVC":
        from ..models.svc import SVC
        from ..utils.data import MinMaxScaler

        t0 = time.perf_counter()
        if self.rank is not None:
            out = self.rank.fit(X, y, self.params)
            dev = f"cuda:{self.rank.device_index}"
        else:
            g = self.group or DsmoGroup.shared(self.world, self.rehearsal)
            out = g.fit(X, y, self.params, trace_cap)
            dev = "cuda:0"
        a = out["alpha"]
        y = np.ascontiguousarray(y, dtype=np.int32)
        sup = np.flatnonzero(a > self.params.sv_tol).astype(np.int64)
        p = self.params
        m = SVC(C=p.C, gamma=p.gamma, tol=p.tau, eps=p.eps, sv_tol=p.sv_tol, max_iter=p.max_iter, device=dev)
        m.scaler_ = MinMaxScaler(out["mn"], out["mx"])
        m.alpha_, m.support_ = a, sup
        m.support_labels_ = y[sup].astype(np.int32)
        m.dual_coef_ = a[sup] * y[sup]
        m.b_, m.intercept_ = out["b"], -out["b"]
        m.n_iter_, m.stop_reason_ = out["iterations"], out["stop_reason"]
        X = np.asarray(X)
        if X.dtype == np.uint8:
            m._device_model_from_u8(X[sup], dev)
        else:  # pixel values held as FP64 (validated integers): widened on the host
            m.support_vectors_ = m.scaler_.transform(X[sup])
            m._upload_model(dev)
        self.model_ = m
        self.alpha_, self.support_, self.b_ = a, sup, out["b"]
        self.n_iter_, self.stop_reason_ = out["iterations"], out["stop_reason"]
        self.trace_ = out.get("trace")
        self.shape_ = out["shape"]
        self.timings_ = out["timings_ms"]
        self.fit_time_ = time.perf_counter() - t0
        return self

    def decision_function(self, X) -> np.ndarray:
        return self.model_.decision_function(X)

    def predict(self, X) -> np.ndarray:
        return self.model_.predict(X)

    def score(self, X, y) -> float:
        return self.model_.score(X, y)


class DsmoRank:
    """This process's team of a per-process distributed SMO (one rank per GPU under torchrun): the
    receive arrays travel as IPC handles over the launcher's process group, each fit is prepare on
    every rank, a barrier, solve on every rank, and the alpha slices are summed to every rank (the
    other entries of a slice are zero, so the sum is exact)."""

    device = "cuda"

    def __init__(self, device: int, world: int, rank: int, timeout_s: float = 60.0):
        self.device_index, self.world, self.rank = int(device), int(world), int(rank)
        self.handle = N.hip().svmd_dsmo_rank_create(self.device_index, self.world, self.rank, float(timeout_s))
        if not self.handle:
            raise N.NativeError(N.last_error())

    def export_handle(self) -> bytes:
        nb = int(N.hip().svmd_dsmo_handle_bytes())
        buf = np.zeros(nb, dtype=np.uint8)
        N.check(N.hip().svmd_dsmo_rank_handle(self.handle, N.ptr(buf), nb), "svmd_dsmo_rank_handle")
        return buf.tobytes()

    def connect(self, handles) -> None:
        allh = np.frombuffer(b"".join(handles), dtype=np.uint8).copy()
        N.check(N.hip().svmd_dsmo_rank_connect(self.handle, N.ptr(allh)), "svmd_dsmo_rank_connect")

    @classmethod
    def from_torch_dist(cls, device: int, timeout_s: float = 60.0, group=None) -> "DsmoRank":
        """Collective over an initialised torch.distributed group (any backend, e.g. gloo)."""
        import torch.distributed as dist

        r = cls(device, dist.get_world_size(group), dist.get_rank(group), timeout_s)
        handles = [None] * r.world
        dist.all_gather_object(handles, r.export_handle(), group=group)
        r.connect(handles)
        return r

    def fit(self, X: np.ndarray, y: np.ndarray, params: Optional[SVMParams] = None, group=None) -> dict:
        """Collective.  Every rank calls the same collectives whatever fails, and every rank raises
        when any rank failed (so a caller can fall back together)."""
        import torch
        import torch.distributed as dist

        from ..utils.data import check_labels, pixel_rows

        p = (params or SVMParams()).to_struct()
        lib, err = N.hip(), ""
        ok = torch.ones(1, dtype=torch.int32)
        try:  # a bad input on any rank fails every rank through the agreement below, not a hang
            X = pixel_rows(X, "the distributed SMO")
            n, d = X.shape
            y = check_labels(y, n)
        except ValueError as e:
            ok[0], err = 0, str(e)
            X = np.zeros((0, 1), dtype=np.uint8)
            n, d = 0, 1
        if ok[0] and lib.svmd_dsmo_rank_prepare(self.handle, N.ptr(X), 1, N.ptr(y), n, d, ctypes.byref(p)) != 0:
            ok[0], err = 0, N.last_error()
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)  # also the launch barrier
        if not ok[0]:  # every rank learns it here and raises: no collective of mismatched sizes follows
            raise (ValueError if err.startswith(("the distributed", "y must", "labels")) else N.NativeError)(
                f"distributed SMO failed on some rank ({err or 'another rank'})")
        alpha = np.zeros(n, dtype=np.float64)
        r = N.SvmResult()
        tm = np.zeros(4, dtype=np.float64)
        shape = np.zeros(4, dtype=np.int32)
        mn, mx = np.empty(d), np.empty(d)
        rng = np.zeros(2, dtype=np.int64)
        if ok[0]:
            if lib.svmd_dsmo_rank_solve(self.handle, N.ptr(alpha), ctypes.byref(r), N.ptr(tm), N.ptr(shape), N.ptr(mn),
                                        N.ptr(mx), N.ptr(rng)) != 0:
                ok[0], err = 0, N.last_error()
        at = torch.from_numpy(alpha)
        dist.all_reduce(at, op=dist.ReduceOp.SUM, group=group)
        # every team must have run the identical solve: compare (iterations, b) across ranks
        key = torch.tensor([float(r.iterations), float(r.b), float(ok[0])], dtype=torch.float64)
        lo, hi = key.clone(), key.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
        if lo[2] < 1:
            raise N.NativeError(f"distributed SMO failed on some rank ({err or 'another rank'})")
        if not torch.equal(lo[:2], hi[:2]):
            raise N.NativeError("distributed SMO: ranks disagree on iterations / b")
        return {"alpha": at.numpy(), "iterations": int(r.iterations), "b": float(r.b),
                "stop_reason": N.STOP_NAMES.get(int(r.stop_reason), str(r.stop_reason)), "mn": mn, "mx": mx,
                "timings_ms": {"upload_minmax_ms": float(tm[0]), "quantise_slab_ms": float(tm[1]),
                               "smo_ms": float(tm[2]), "total_ms": float(tm[3])},
                "shape": {"threads": int(shape[0]), "points_per_thread": int(shape[1]),
                          "workgroups_per_team": int(shape[2]), "records_per_lane": int(shape[3])},
                "slice": (int(rng[0]), int(rng[1]))}

    def close(self) -> None:
        if getattr(self, "handle", None):
            N.hip().svmd_dsmo_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
