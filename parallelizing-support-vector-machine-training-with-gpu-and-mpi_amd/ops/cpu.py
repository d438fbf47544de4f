"""CPU ops backed by the native core (libsvm355_core.so): the reference-exact oracle.

These implement main3.cpp's serial semantics (SMO_train :162-294, warm start
mpi_svm_main3.cpp:155-290, predict :391-402).  ``n_threads > 1`` parallelises the O(n) loops
without changing any result bit.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from .. import _native as N
from ..utils.config import SVMParams
from .device import SMOResult


def _c64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def _c32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


def _start(alpha, n: int) -> np.ndarray:
    """The solver's alpha buffer: zeros, or a copy of the warm start, which must have n entries (the native
    solvers read n of them)."""
    if alpha is None:
        return np.zeros(n)
    if np.shape(alpha) != (n,):
        raise ValueError(f"alpha must have shape ({n},), got {np.shape(alpha)}")
    return np.array(alpha, dtype=np.float64, copy=True)


def _gram_shape(K: np.ndarray, n: int) -> None:
    if K.ndim != 2 or K.shape[0] < n or K.shape[1] < n:
        raise ValueError(f"K must be at least ({n}, {n}) for {n} labels, got {K.shape}")


def smo_train(X: np.ndarray, y: np.ndarray, params: SVMParams, alpha: Optional[np.ndarray] = None,
              warm: bool = False, trace_cap: int = 0, verbose: int = 0
              ) -> Tuple[np.ndarray, SMOResult, Optional[np.ndarray]]:
    """SMO on (already scaled) rows X with labels y in {+1,-1}.  Returns (alpha, result, trace)."""
    X = _c64(X)
    y = _c32(y)
    n, d = X.shape
    if y.shape != (n,):
        raise ValueError(f"y must have shape ({n},), got {y.shape}")
    a = _start(alpha, n)
    r = N.SvmResult()
    trace = np.zeros((trace_cap, 2), dtype=np.int64) if trace_cap > 0 else None
    p = params.to_struct(verbose)
    N.check(N.core().svm_smo_train(N.ptr(X), N.ptr(y), n, d, N.ptr(a), int(warm), ctypes.byref(p), ctypes.byref(r),
                                   N.ptr(trace) if trace is not None else None, trace_cap), "svm_smo_train")
    res = SMOResult.from_struct(r)
    if trace is not None:
        trace = trace[: max(0, min(trace_cap, res.iterations - 1))]
    return a, res, trace


def smo_train_gram(K: np.ndarray, y: np.ndarray, params: SVMParams, alpha: Optional[np.ndarray] = None,
                   warm: bool = False, trace_cap: int = 0) -> Tuple[np.ndarray, SMOResult, Optional[np.ndarray]]:
    K = _c64(K)
    y = _c32(y)
    n = y.shape[0]
    _gram_shape(K, n)
    a = _start(alpha, n)
    r = N.SvmResult()
    trace = np.zeros((trace_cap, 2), dtype=np.int64) if trace_cap > 0 else None
    p = params.to_struct()
    N.check(N.core().svm_smo_train_gram(N.ptr(K), K.shape[1], N.ptr(y), n, N.ptr(a), int(warm), ctypes.byref(p),
                                        ctypes.byref(r), N.ptr(trace) if trace is not None else None, trace_cap),
            "svm_smo_train_gram")
    res = SMOResult.from_struct(r)
    if trace is not None:
        trace = trace[: max(0, min(trace_cap, res.iterations - 1))]
    return a, res, trace


def decomp_train_gram(K: np.ndarray, y: np.ndarray, params: SVMParams, alpha: Optional[np.ndarray] = None,
                      q: int = 1024, tau_frac: float = 0.1, inner_wss: int = 3, trace_cap: int = 0,
                      snapshots: bool = False):
    """CPU oracle of the device decomposition solver (csrc/core/decomp_cpu.cpp) on a kernel matrix K.
    alpha given = warm start.  Returns (alpha, SMOResult, stats dict, N.DecompTrace or None)."""
    K = _c64(K)
    y = _c32(y)
    n = y.shape[0]
    _gram_shape(K, n)
    a = _start(alpha, n)
    r = N.SvmResult()
    st = (ctypes.c_int64 * 16)()
    tr = N.DecompTrace(trace_cap, n if snapshots else 0) if trace_cap > 0 else None
    p = params.to_struct()
    N.check(N.core().svm_decomp_train_gram(N.ptr(K), K.shape[1], N.ptr(y), n, N.ptr(a), int(alpha is not None),
                                           ctypes.byref(p), int(q), float(tau_frac), int(inner_wss), ctypes.byref(r),
                                           st, ctypes.byref(tr.struct) if tr is not None else None),
            "svm_decomp_train_gram")
    return a, SMOResult.from_struct(r), _decomp_stats(st), tr


def _decomp_stats(st) -> dict:
    return {"outer_iterations": int(st[0]), "inner_iterations": int(st[1]), "working_set": int(st[2]),
            "solve_us": int(st[3]), "update_columns": int(st[4]), "chain_iterations": int(st[13]),
            **N.shrink_stats(st)}


def decomp_train_gram_dist(K: np.ndarray, y: np.ndarray, params: SVMParams, world: int = 1, comm=None,
                           alpha: Optional[np.ndarray] = None, q: int = 1024, tau_frac: float = 0.1,
                           inner_wss: int = 3, comm_timeout_s: float = 120.0):
    """The distributed form of ``decomp_train_gram`` (decomp.hip's world > 1 solve on the CPU oracle):
    ``comm`` = a ``HostCommRank`` (this process's rank over a gloo group, torchrun), or ``world``
    thread-ranks of this process over the strict loopback transport.  Every rank owns 1/world of the
    selection blocks and of f and all-gathers its candidate records once per outer iteration; for world
    dividing 8 the result is ``decomp_train_gram``'s bit for bit.  Returns (alpha, SMOResult, stats)."""
    K = _c64(K)
    y = _c32(y)
    n = y.shape[0]
    _gram_shape(K, n)
    a = _start(alpha, n)
    r = N.SvmResult()
    st = (ctypes.c_int64 * 16)()
    p = params.to_struct()
    if comm is not None:
        comm.error = None
        rc = N.core().svm_decomp_rank_train_gram(ctypes.addressof(comm.comm), N.ptr(K), K.shape[1], N.ptr(y), n,
                                                 N.ptr(a), int(alpha is not None), ctypes.byref(p), int(q),
                                                 float(tau_frac), int(inner_wss), ctypes.byref(r), st)
        if rc != 0 and comm.error is not None:
            raise N.NativeError(f"{N.last_error()} (collective error: {comm.error!r})") from comm.error
        N.check(rc, "svm_decomp_rank_train_gram")
    else:
        N.check(N.core().svm_decomp_group_train_gram(int(world), N.ptr(K), K.shape[1], N.ptr(y), n, N.ptr(a),
                                                     int(alpha is not None), ctypes.byref(p), int(q), float(tau_frac),
                                                     int(inner_wss), ctypes.byref(r), st, float(comm_timeout_s)),
                "svm_decomp_group_train_gram")
    return a, SMOResult.from_struct(r), _decomp_stats(st)


def rbf_matrix(A: np.ndarray, B: np.ndarray, gamma: float, n_threads: int = 0) -> np.ndarray:
    """Reference-exact RBF kernel matrix (direct sum of squared differences)."""
    A = _c64(A)
    B = _c64(B)
    K = np.empty((A.shape[0], B.shape[0]))
    N.check(N.core().svm_rbf_matrix(N.ptr(A), A.shape[0], N.ptr(B), B.shape[0], A.shape[1], float(gamma), N.ptr(K),
                                    int(n_threads)), "svm_rbf_matrix")
    return K


def decision(Xs: np.ndarray, ys: np.ndarray, alphas: np.ndarray, Xq: np.ndarray, gamma: float, b: float,
             n_threads: int = 0) -> np.ndarray:
    Xs = _c64(Xs).reshape(-1, Xq.shape[1])
    ys = _c32(ys)
    alphas = _c64(alphas)
    Xq = _c64(Xq)
    out = np.empty(Xq.shape[0])
    N.check(N.core().svm_decision(N.ptr(Xs), N.ptr(ys), N.ptr(alphas), Xs.shape[0], N.ptr(Xq), Xq.shape[0],
                                  Xq.shape[1], float(gamma), float(b), N.ptr(out), int(n_threads)), "svm_decision")
    return out


def sv_indices(alpha: np.ndarray, tol: float = 1e-8) -> np.ndarray:
    alpha = _c64(alpha)
    out = np.empty(alpha.shape[0], dtype=np.int64)
    k = N.core().svm_sv_indices(N.ptr(alpha), alpha.shape[0], float(tol), N.ptr(out))
    return out[:k].copy()
