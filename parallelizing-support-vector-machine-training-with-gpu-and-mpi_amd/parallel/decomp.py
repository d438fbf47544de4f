"""Distributed working-set decomposition SMO over the GPUs of one node (``--parallel decomp``;
csrc/hip/decomp.hip + the group / rank entry points of csrc/hip/cascade_dev.hip).

The one-GPU decomposition solver (``SVC(solver="decomp")``) spends its outer iterations on three
kinds of work: choosing the working set (top violators per block of points), solving it (one
workgroup, latency-bound), and updating f for all n points (an int8-MFMA GEMV over the points whose
alpha moved).  The first and last scale with n; the middle does not.  Here every GPU:

- holds all n rows (uint8 pixels quantised on its own device: exact-integer kernel values; or FP64
  rows min-max scaled on it: FP64-MFMA kernel values for real-valued data), the labels and a replica of
  alpha;
- owns a contiguous range of the selection's blocks and keeps f for those points only;
- selects its blocks' candidates, and ONE all-gather per outer iteration (RCCL ``ncclAllGather``
  over xGMI, 16-byte records: id and f) gives every GPU the same candidate list;
- builds the same working set, runs the same inner solve on the same inputs (so the alpha replicas
  stay identical without any exchange), and updates f for its own points.

The selection's block partition is global and a multiple of 8 blocks, so with 1, 2, 4 or 8 GPUs the
trajectory -- every working set, every alpha, b and the iteration counts -- equals the one-GPU
decomposition solver's (tests/test_gpu_decomp.py).  It pays where the GEMV and the selection
dominate: large n (see README "Distributed decomposition").

Launch forms: a ``DeviceGroup`` of this process (thread ranks, ``ncclCommInitAll``; or
``transport="loopback"``: P ranks rehearsed on the visible GPU), or one rank per process under
torchrun: ``RcclRank`` (``ncclCommInitRank``) or ``HostCommDeviceRank`` (the same driver with the
candidate all-gather over a gloo group, device buffers staged through the host: P processes may share
ONE GPU, so the per-process path runs at world > 1 on a one-GPU box).  On the CPU the same solve runs
on the decomposition oracle (``HostCommRank`` under torchrun, or ``transport="cpu"`` thread ranks):
the multi-process twin the CPU tests launch.
"""
from __future__ import annotations

import ctypes
import time
from typing import Optional

import numpy as np

from .. import _native as N
from ..utils.config import SVMParams
from ..utils.trace import trace_range


def _rows(X) -> tuple:
    """(rows, is_u8): integer pixel rows as uint8 (the exact-integer path, 8x less host-to-device traffic),
    anything else as C-contiguous FP64 (min-max scaled on the GPUs; real-valued data train with FP64-MFMA
    kernel values, mpi_svm_main2.cpp:316-402 / mpi_svm_main3.cpp:433-518 partition double rows)."""
    from ..utils.data import check_finite_bounds, compact_pixels

    Xc = compact_pixels(X)
    if Xc is not None and Xc.ndim == 2:
        return np.ascontiguousarray(Xc), True
    X = np.ascontiguousarray(X, dtype=np.float64)
    if X.ndim != 2:
        raise ValueError("X must be (n, d)")
    check_finite_bounds(X.min(0), X.max(0))
    return X, False


def _fit_native(fn, handle, X: np.ndarray, y: np.ndarray, params: SVMParams, q: int, world: int) -> dict:
    from ..utils.data import check_labels

    n, d = X.shape
    y = check_labels(y, n)
    alpha = np.empty(n, dtype=np.float64)
    mm = np.empty(2 * d, dtype=np.float64)
    r = N.SvmResult()
    st = (ctypes.c_int64 * 16)()
    ms = np.zeros(max(world, 1), dtype=np.float64)
    p = params.to_struct()
    t0 = time.perf_counter()
    with trace_range(f"svm355.decomp.solve world={world} n={n}"):
        N.check(fn(handle, N.ptr(X), N.ptr(y), n, d, ctypes.byref(p), int(q), N.ptr(alpha), ctypes.byref(r), st,
                   N.ptr(ms), N.ptr(mm)), fn.__name__)
    wall = (time.perf_counter() - t0) * 1e3
    return {"alpha": alpha, "b": float(r.b), "b_high": float(r.b_high), "b_low": float(r.b_low),
            "iterations": int(r.iterations), "stop_reason": N.STOP_NAMES.get(int(r.stop_reason), str(r.stop_reason)),
            "n_sv": int(r.n_sv), "mn": mm[:d].copy(), "mx": mm[d:].copy(),
            "stats": {"outer_iterations": int(st[0]), "inner_iterations": int(st[1]), "working_set": int(st[2]),
                      "solve_us": int(st[3]), "update_columns": int(st[4]), "inner_threads": int(st[5]),
                      **N.shrink_stats(st)},
            "rank_ms": [float(x) for x in ms[:world]], "wall_ms": wall}


def cpu_fit(X: np.ndarray, y: np.ndarray, params: Optional[SVMParams] = None, q: int = 1024, world: int = 1,
            comm=None) -> dict:
    """The same distributed solve on the CPU oracle (csrc/core/decomp_cpu.cpp): ``comm`` = this process's
    ``HostCommRank`` (torchrun over gloo: the CPU twin of the per-process GPU rank), else ``world``
    thread-ranks of this process.  Every rank holds the whole reference-exact kernel matrix of the
    min-max scaled rows (``ops.cpu.rbf_matrix``; small n only), owns 1/world of the selection blocks and
    of f, and all-gathers its candidate records once per outer iteration."""
    from ..ops import cpu as C
    from ..utils.data import MinMaxScaler, check_labels

    params = params or SVMParams()
    X = np.asarray(X)
    n, d = X.shape
    if n > 20000:
        raise ValueError(f"the CPU decomposition oracle holds the whole {n} x {n} kernel matrix: n <= 20000")
    y = check_labels(y, n)
    sc = MinMaxScaler().fit(X)
    Xs = sc.transform(X)
    t0 = time.perf_counter()
    with trace_range(f"svm355.decomp.cpu world={comm.world if comm is not None else world} n={n}"):
        K = C.rbf_matrix(Xs, Xs, params.gamma, params.n_threads)
        a, r, st = C.decomp_train_gram_dist(K, y, params, world=world, comm=comm, q=q,
                                            comm_timeout_s=getattr(comm, "timeout_s", 120.0))
    wall = (time.perf_counter() - t0) * 1e3
    return {"alpha": a, "b": r.b, "b_high": r.b_high, "b_low": r.b_low, "iterations": r.iterations,
            "stop_reason": r.stop_reason, "n_sv": int(np.count_nonzero(a > params.sv_tol)), "mn": sc.min_,
            "mx": sc.max_, "stats": {**st, "inner_threads": 0}, "rank_ms": [wall], "wall_ms": wall, "rows": Xs}


def group_fit(group, X: np.ndarray, y: np.ndarray, params: Optional[SVMParams] = None, q: int = 1024) -> dict:
    """One distributed decomposition solve over a ``DeviceGroup`` (its ranks are this process's
    threads; RCCL or the loopback rehearsal)."""
    lib = N.hip()
    X, u8 = _rows(X)
    fn = lib.svmd_cascade_group_decomp if u8 else lib.svmd_cascade_group_decomp_rows
    out = _fit_native(fn, group.handle, X, y, params or SVMParams(), q, group.world)
    waits = np.zeros(group.world)
    if int(lib.svmd_cascade_group_decomp_waits(group.handle, N.ptr(waits), waits.size)) == group.world:
        out["host_wait_ms"] = [round(float(v), 3) for v in waits]
    buf = np.zeros(4 + 2 * group.world)
    k = int(lib.svmd_cascade_group_decomp_solo(group.handle, N.ptr(buf), buf.size))
    if k:  # a loopback rehearsal with SVM355_CASCADE_SERIAL_SOLVES=1: every rank's device work timed alone
        out["solo"] = {"critical_path_ms": float(buf[0]), "select_ms": float(buf[1]), "rest_ms": float(buf[2]),
                       "outer_iterations": int(buf[3]),
                       "rank_select_ms": [float(v) for v in buf[4:k:2]], "rank_rest_ms": [float(v) for v in buf[5:k:2]]}
    return out


def rank_fit(rank, X: np.ndarray, y: np.ndarray, params: Optional[SVMParams] = None, q: int = 1024) -> dict:
    """This process's rank of a distributed decomposition solve (every rank passes all rows)."""
    lib = N.hip()
    X, u8 = _rows(X)
    fn = lib.svmd_cascade_rank_decomp if u8 else lib.svmd_cascade_rank_decomp_rows
    out = _fit_native(fn, rank.handle, X, y, params or SVMParams(), q, 1)
    out["host_wait_ms"] = [round(float(lib.svmd_cascade_rank_decomp_wait(rank.handle)), 3)]
    return out


class DistributedDecompSVC:
    """Estimator over a ``DeviceGroup`` or an ``RcclRank``: ``fit`` / ``decision_function`` /
    ``predict`` / ``score``; the fitted model is an ``SVC`` on this process's GPU."""

    def __init__(self, world: int = 1, transport: str = "auto", C: float = 10.0, gamma: float = 0.00125,
                 tol: float = 1e-5, eps: float = 1e-12, sv_tol: float = 1e-8, max_iter: int = 100000,
                 working_set: int = 1024, group=None, rank=None):
        self.params = SVMParams(C=C, gamma=gamma, tau=tol, eps=eps, sv_tol=sv_tol, max_iter=max_iter)
        self.world, self.transport, self.group, self.rank = world, transport, group, rank
        self.working_set = int(working_set)

    def fit(self, X: np.ndarray, y: np.ndarray) -> "DistributedDecompSVC":
        from ..models.svc import SVC
        from ..utils.data import MinMaxScaler
        from .rccl import DeviceGroup

        t0 = time.perf_counter()
        if self.rank is not None and self.rank.device == "cpu":  # HostCommRank: the CPU twin under torchrun
            out = cpu_fit(X, y, self.params, self.working_set, comm=self.rank)
            dev = "cpu"
        elif self.rank is None and self.transport == "cpu":  # thread ranks on the CPU oracle
            out = cpu_fit(X, y, self.params, self.working_set, world=self.world)
            dev = "cpu"
        elif self.rank is not None:
            out = rank_fit(self.rank, X, y, self.params, self.working_set)
            dev = f"cuda:{self.rank.device}"
        else:
            g = self.group or DeviceGroup.shared(self.world, self.transport)
            out = group_fit(g, X, y, self.params, self.working_set)
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
        with trace_range("svm355.decomp.model"):
            if dev == "cpu":
                m.support_vectors_ = out["rows"][sup]
            elif X.dtype == np.uint8:
                m._device_model_from_u8(X[sup], dev)
            else:  # FP64 rows (real-valued, or pixel values as doubles): scaled on the host
                m.support_vectors_ = m.scaler_.transform(X[sup])
                m._upload_model(dev)
        self.model_ = m
        self.alpha_, self.support_, self.b_ = a, sup, out["b"]
        self.n_iter_, self.stop_reason_ = out["iterations"], out["stop_reason"]
        self.stats_ = out["stats"]
        self.rank_ms_ = out["rank_ms"]
        self.solo_ = out.get("solo")  # per-rank solo timing of a one-GPU rehearsal (None otherwise)
        self.host_wait_ms_ = out.get("host_wait_ms")  # per-rank host time blocked in the per-batch waits
        self.timings_ = {"solve_ms": out["stats"]["solve_us"] / 1e3, "native_ms": out["wall_ms"],
                         **out["stats"]}
        self.fit_time_ = time.perf_counter() - t0
        return self

    def decision_function(self, X) -> np.ndarray:
        return self.model_.decision_function(X)

    def predict(self, X) -> np.ndarray:
        return self.model_.predict(X)

    def score(self, X, y) -> float:
        return self.model_.score(X, y)
