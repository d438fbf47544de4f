"""Device ops on PyTorch-ROCm tensors backed by the hand-written gfx950 kernels (libsvm355_hip.so).

Every op enqueues on the tensor's device behind PyTorch's current stream (the device context is
re-bound to ``torch.cuda.current_stream()`` on every call), so these compose with ordinary torch
code.  Feature matrices are ``(n, ld)`` float64 with ``ld = padded_dim(d)`` (multiple of 16,
zero-padded).  A missing or unloadable device library raises :class:`svm355._native.NativeError`:
there is no eager/torch fallback for any of these kernels.

Reference kernels these replace (/root/reference/code/gpu_svm_main3.cu): find_min_max :62-95,
scale_features :100-116, calc_kernel_matrix :137-147, init/WSS/update kernels :152-272,
predict + reduce_sum :277-315.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np
import torch

from .. import _native as N
from ..utils.config import SVMParams


@dataclass
class SMOResult:
    iterations: int
    b: float
    b_high: float
    b_low: float
    stop_reason: str
    n_sv: int
    seconds: float

    @classmethod
    def from_struct(cls, r: N.SvmResult) -> "SMOResult":
        return cls(int(r.iterations), float(r.b), float(r.b_high), float(r.b_low),
                   N.STOP_NAMES.get(int(r.stop_reason), str(r.stop_reason)), int(r.n_sv), float(r.seconds))


class DeviceContext:
    """One native device context (private HIP stream + workspace) per GPU per host thread
    (thread-ranks sharing a GPU must not share a workspace).  Contexts live in thread-local storage:
    when a worker thread ends, its contexts (and their library-owned Gram) are destroyed with it."""

    _tls = threading.local()

    def __init__(self, index: int):
        self.index = index
        self.lib = N.hip()
        with torch.cuda.device(index):
            self.handle = self.lib.svmd_create(index)
        if not self.handle:
            raise N.NativeError(f"svmd_create({index}) failed: {N.last_error()}")

    def __del__(self):
        h, self.handle = getattr(self, "handle", None), None
        if h:
            try:
                self.lib.svmd_destroy(h)
            except Exception:  # interpreter shutdown
                pass

    @classmethod
    def get(cls, device) -> "DeviceContext":
        index = torch.device(device).index
        if index is None:
            index = torch.cuda.current_device()
        ctxs = getattr(cls._tls, "ctxs", None)
        if ctxs is None:
            ctxs = cls._tls.ctxs = {}
        ctx = ctxs.get(index)
        if ctx is None:
            ctx = ctxs[index] = DeviceContext(index)
        return ctx

    def bind(self) -> int:
        stream = torch.cuda.current_stream(self.index)
        N.check(self.lib.svmd_set_stream(self.handle, stream.cuda_stream), "svmd_set_stream")
        return self.handle


def _ctx_for(t: torch.Tensor) -> DeviceContext:
    if not t.is_cuda:
        raise ValueError("device op needs a GPU tensor")
    return DeviceContext.get(t.device)


def _check_rows(X: torch.Tensor, name: str = "X") -> None:
    if X.dtype != torch.float64 or X.dim() != 2 or not X.is_contiguous():
        raise ValueError(f"{name} must be a contiguous 2-D float64 tensor, got {X.dtype} {tuple(X.shape)}")
    if X.shape[1] % 16:
        raise ValueError(f"{name} row length must be a multiple of 16 (use padded_dim), got {X.shape[1]}")


def padded_dim(d: int) -> int:
    return (int(d) + 15) // 16 * 16


def available() -> bool:
    """True if a GPU is visible and the device library loads."""
    if not torch.cuda.is_available():
        return False
    N.hip()
    return True


def device_empty(shape, dtype, device) -> torch.Tensor:
    """``torch.empty`` for the library's large device buffers.  On an out-of-memory error the memory the
    library itself holds outside PyTorch's allocator -- the Gram and the row-cache / column-cache slab
    its contexts keep between fits, the grow-only Gram buffers (``release_gram_buffers``), and the
    one-vs-rest pool threads' column-cache slabs (``models.multiclass.release_solver_caches``) -- is handed
    back and the allocation retried once: a cache kept for speed never makes a later allocation fail
    (ADVICE r4, r5).""" 
    try:
        return torch.empty(shape, dtype=dtype, device=device)
    except torch.OutOfMemoryError:
        release_gram_buffers()
        # and the one-vs-rest pool threads' column-cache slabs (their contexts are not this thread's)
        from ..models.multiclass import release_solver_caches

        release_solver_caches(timeout_s=1.0)
        torch.cuda.empty_cache()
        return torch.empty(shape, dtype=dtype, device=device)


def upload_rows(X: np.ndarray, device, ld: Optional[int] = None) -> torch.Tensor:
    """Host (n, d) rows -> device (n, ld) zero-padded FP64 rows.

    float rows go over PCIe as FP64 (hipMemcpy2DAsync).  uint8 rows (pixel data, see
    ``utils.data.compact_pixels``) go over as bytes, 8x less H2D traffic, and are widened to FP64 on
    the device (every value is exact), so everything downstream is identical."""
    if isinstance(X, np.ndarray) and X.dtype == np.uint8:
        X = np.ascontiguousarray(X)
        n, d = X.shape
        ld = padded_dim(d) if ld is None else ld
        out = device_empty((n, ld), torch.float64, device)
        ctx = DeviceContext.get(out.device)
        N.check(ctx.lib.svmd_upload_rows_u8(ctx.bind(), N.ptr(X), n, d, N.ptr(out), ld), "svmd_upload_rows_u8")
        return out
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, d = X.shape
    ld = padded_dim(d) if ld is None else ld
    out = device_empty((n, ld), torch.float64, device)
    ctx = DeviceContext.get(out.device)
    N.check(ctx.lib.svmd_upload_rows(ctx.bind(), N.ptr(X), n, d, N.ptr(out), ld), "svmd_upload_rows")
    return out


def minmax(X: torch.Tensor, d: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Column min/max of the first d columns (one streaming pass, per-block partials)."""
    _check_rows(X)
    ctx = _ctx_for(X)
    mn = torch.empty(d, dtype=torch.float64, device=X.device)
    mx = torch.empty(d, dtype=torch.float64, device=X.device)
    N.check(ctx.lib.svmd_minmax(ctx.bind(), N.ptr(X), X.shape[0], d, X.shape[1], N.ptr(mn), N.ptr(mx)),
            "svmd_minmax")
    return mn, mx


def minmax_scale_(X: torch.Tensor, d: int, mn: Optional[torch.Tensor] = None,
                  mx: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """In-place min-max scaling of the first d columns; returns (min, max, squared row norms).

    With mn/mx given they are used as-is (test data scaled with training statistics)."""
    _check_rows(X)
    ctx = _ctx_for(X)
    n = X.shape[0]
    use_given = mn is not None
    if not use_given:  # one buffer: the caller reads both bounds back with one copy (torch.cat-free)
        mm = torch.empty(2 * d, dtype=torch.float64, device=X.device)
        mn, mx = mm[:d], mm[d:]
    sqn = torch.empty(n, dtype=torch.float64, device=X.device)
    N.check(ctx.lib.svmd_preprocess(ctx.bind(), N.ptr(X), n, d, X.shape[1], N.ptr(mn), N.ptr(mx), N.ptr(sqn),
                                    int(use_given)), "svmd_preprocess")
    return mn, mx, sqn


def row_norms(X: torch.Tensor, d: Optional[int] = None) -> torch.Tensor:
    _check_rows(X)
    ctx = _ctx_for(X)
    d = X.shape[1] if d is None else d
    out = torch.empty(X.shape[0], dtype=torch.float64, device=X.device)
    N.check(ctx.lib.svmd_row_norms(ctx.bind(), N.ptr(X), X.shape[0], d, X.shape[1], N.ptr(out)), "svmd_row_norms")
    return out


def rbf_gram(A: torch.Tensor, nA: torch.Tensor, B: torch.Tensor, nB: torch.Tensor, gamma: float,
             symmetric: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K[i, j] = exp(-gamma ||A_i - B_j||^2) on MFMA f64 tiles (diagonal forced to 1 if symmetric)."""
    _check_rows(A, "A")
    _check_rows(B, "B")
    if A.shape[1] != B.shape[1]:
        raise ValueError("A and B row lengths differ")
    m, n = A.shape[0], B.shape[0]
    if out is None:
        ldk = (n + 1) // 2 * 2
        out = torch.empty((m, ldk), dtype=torch.float64, device=A.device)
    ctx = _ctx_for(A)
    N.check(ctx.lib.svmd_rbf_gram(ctx.bind(), N.ptr(A), N.ptr(nA), m, A.shape[1], N.ptr(B), N.ptr(nB), n,
                                  B.shape[1], A.shape[1], float(gamma), N.ptr(out), out.stride(0), int(symmetric)),
            "svmd_rbf_gram")
    return out


def smo(K: torch.Tensor, y: torch.Tensor, alpha: torch.Tensor, params: SVMParams, warm: bool = False,
        n: Optional[int] = None, trace_cap: int = 0) -> Tuple[SMOResult, Optional[np.ndarray]]:
    """Device-resident SMO on a kernel matrix; alpha is updated in place."""
    n = K.shape[0] if n is None else n
    if y.dtype != torch.int32 or alpha.dtype != torch.float64:
        raise ValueError("y must be int32 (+-1) and alpha float64")
    ctx = _ctx_for(K)
    r = N.SvmResult()
    trace = np.zeros((max(trace_cap, 0), 2), dtype=np.int64) if trace_cap > 0 else None
    p = params.to_struct()
    N.check(ctx.lib.svmd_smo(ctx.bind(), N.ptr(K), K.stride(0), N.ptr(y), n, N.ptr(alpha), int(warm),
                             ctypes.byref(p), ctypes.byref(r), N.ptr(trace) if trace is not None else None,
                             trace_cap), "svmd_smo")
    res = SMOResult.from_struct(r)
    if trace is not None:
        trace = trace[: max(0, min(trace_cap, res.iterations - 1))]
    return res, trace


def smo_multi(K: torch.Tensor, Y: torch.Tensor, A: torch.Tensor, params: SVMParams,
              n: Optional[int] = None) -> Tuple[List[SMOResult], bool]:
    """``nclass`` cold-start SMO solves on one resident Gram (one-vs-rest): Y (nclass, n) int32 +-1,
    A (nclass, n) float64 receives the alphas.  The classes run concurrently, one XCD-local team per
    XCD (smo.hip, smo_multi_kernel); each result equals the single solve's bit for bit.
    Returns (results, batched) — batched False when the solves ran one by one."""
    n = K.shape[0] if n is None else n
    if Y.dtype != torch.int32 or A.dtype != torch.float64 or Y.shape != A.shape or Y.shape[1] != n:
        raise ValueError("Y must be (nclass, n) int32 and A (nclass, n) float64")
    if not (Y.is_contiguous() and A.is_contiguous()):
        raise ValueError("Y and A must be contiguous (class-major)")
    nclass = Y.shape[0]
    ctx = _ctx_for(K)
    rs = (N.SvmResult * nclass)()
    batched = ctypes.c_int32(0)
    p = params.to_struct()
    N.check(ctx.lib.svmd_smo_multi(ctx.bind(), N.ptr(K), K.stride(0), N.ptr(Y), n, nclass, N.ptr(A),
                                   ctypes.byref(p), rs, ctypes.byref(batched)), "svmd_smo_multi")
    return [SMOResult.from_struct(r) for r in rs], bool(batched.value)


GRAM_MODES = {"auto": 0, "fp64": 1, "int": 2}


def _host_stats(mn, mx):
    if mn is None or mx is None:
        return None, None, 0
    a = np.ascontiguousarray(mn.detach().cpu().numpy() if isinstance(mn, torch.Tensor) else mn, dtype=np.float64)
    b = np.ascontiguousarray(mx.detach().cpu().numpy() if isinstance(mx, torch.Tensor) else mx, dtype=np.float64)
    return a, b, int(a.shape[0])


_GRAM_TLS = threading.local()  # per host thread: {device index: grow-only Gram buffer}


def _gram_bufs() -> dict:
    bufs = getattr(_GRAM_TLS, "bufs", None)
    if bufs is None:
        bufs = _GRAM_TLS.bufs = {}
    return bufs


def gram_buffer(n: int, device) -> torch.Tensor:
    """(n, ldk) float64 scratch Gram for the library's own transient use (SVC fit, one-vs-rest):
    one grow-only buffer per device per host thread, so repeated fits of the same or smaller size
    never go back to the allocator — a fresh multi-GB device allocation can take hundreds of
    milliseconds.  The view is overwritten by the next call on the same thread.  Buffers live in
    thread-local storage (released when the thread ends) and ``release_gram_buffers()`` drops the
    calling thread's."""
    device = torch.device(device)
    ldk = (n + 1) // 2 * 2
    key = device.index if device.index is not None else torch.cuda.current_device()
    bufs = _gram_bufs()
    buf = bufs.get(key)
    if buf is None or buf.numel() < n * ldk:
        bufs.pop(key, None)
        del buf
        buf = bufs[key] = device_empty(n * ldk, torch.float64, device)
    return buf[: n * ldk].view(n, ldk)


def release_gram_buffers() -> None:
    """Drop the calling thread's cached Gram buffers (``gram_buffer``) and the library-owned device
    memory of its contexts (the row-cache slab and Gram the C ABI keeps between fits, which would
    otherwise hold up to 60 % of the HBM and push later fits onto the slower row cache)."""
    _gram_bufs().clear()
    for ctx in list((getattr(DeviceContext._tls, "ctxs", None) or {}).values()):
        if ctx.handle:
            N.check(ctx.lib.svmd_release_cache(ctx.handle), "svmd_release_cache")


def gram_fits(n: int, device, fraction: float = 0.8) -> bool:
    """Does the full n x n float64 Gram fit in `fraction` of the free device memory?  A row-cache slab
    an earlier fit left in this thread's context counts as free: when the Gram fits only with that
    memory the slab is handed back (it is rebuilt on demand), so it cannot push this fit onto the row
    cache; otherwise it is kept for the next row-cache fit."""
    device = torch.device(device)
    need = n * ((n + 1) // 2 * 2) * 8
    free, _ = torch.cuda.mem_get_info(device)
    avail = free + torch.cuda.memory_reserved(device)
    ctx = (getattr(DeviceContext._tls, "ctxs", None) or {}).get(
        device.index if device.index is not None else torch.cuda.current_device())
    if ctx is None or not ctx.handle or need <= fraction * avail:
        return need <= fraction * avail
    slab = ctypes.c_int64(0)
    N.check(ctx.lib.svmd_cache_bytes(ctx.handle, None, ctypes.byref(slab)), "svmd_cache_bytes")
    if slab.value and need <= fraction * (avail + slab.value):
        N.check(ctx.lib.svmd_release_slab(ctx.handle), "svmd_release_slab")
        return True
    return False


def train(X: torch.Tensor, sqn: torch.Tensor, y: torch.Tensor, alpha: torch.Tensor, params: SVMParams,
          warm: bool = False, K: Optional[torch.Tensor] = None, mn=None, mx=None,
          gram: str = "auto", kcache: str = "auto", cache_bytes: int = 0,
          trace_cap: int = 0) -> Tuple[SMOResult, dict]:
    """RBF kernel + SMO.  Returns (result, timing dict in ms).

    ``mn``/``mx`` are the min/max the rows were scaled with; with them the exact-integer Gram
    (int8 MFMA, igram.hip) runs when the rows are integer-valued pixels (``gram="auto"``),
    ``gram="fp64"`` forces the FP64 MFMA Gram, ``gram="int"`` requires the integer path.
    ``kcache="full"`` stores the whole Gram (into K, allocated by torch if None); ``"rows"`` uses
    the on-demand HBM row cache (rowcache.hip) for problems whose Gram does not fit; ``"auto"``
    picks "full" when the Gram fits in 80% of the free memory."""
    _check_rows(X)
    n = X.shape[0]
    if kcache == "auto":
        kcache = "full" if (K is not None or gram_fits(n, X.device)) else "rows"
    ctx = _ctx_for(X)
    r = N.SvmResult()
    p = params.to_struct()
    a, b, d = _host_stats(mn, mx)
    used = ctypes.c_int32(0)
    trace = np.zeros((max(trace_cap, 0), 2), dtype=np.int64) if trace_cap > 0 else None
    if kcache == "rows":
        import time as _t

        # the row cache sizes itself from the free HBM: hand this thread's scratch Gram back first
        if _gram_bufs().pop(X.device.index, None) is not None:
            torch.cuda.empty_cache()

        t0 = _t.perf_counter()
        N.check(ctx.lib.svmd_train_rows(ctx.bind(), N.ptr(X), N.ptr(sqn) if sqn is not None else None, n, X.shape[1],
                                        X.shape[1], N.ptr(y), N.ptr(alpha), int(warm), ctypes.byref(p),
                                        ctypes.byref(r), N.ptr(a), N.ptr(b), GRAM_MODES[gram], int(cache_bytes),
                                        ctypes.byref(used), N.ptr(trace), max(trace_cap, 0)), "svmd_train_rows")
        tms = (_t.perf_counter() - t0) * 1e3
        res = SMOResult.from_struct(r)
        out = {"gram_ms": 0.0, "smo_ms": tms, "total_ms": tms, "kcache": "rows",
               "gram_path": "int8-exact" if used.value else "fp64"}
        if trace is not None:
            out["trace"] = trace[: max(0, min(trace_cap, res.iterations - 1))]
        return res, out
    if trace_cap > 0:
        raise ValueError("trace_cap is supported by the row-cache path only (use smo() on a Gram)")
    import time as _t

    ta = _t.perf_counter()
    if K is None:
        K = gram_buffer(n, X.device)
    alloc_ms = (_t.perf_counter() - ta) * 1e3
    tm = N.SvmdTiming()
    N.check(ctx.lib.svmd_train_q(ctx.bind(), N.ptr(X), N.ptr(sqn) if sqn is not None else None, n, X.shape[1],
                                 X.shape[1], N.ptr(y), N.ptr(alpha), int(warm), ctypes.byref(p), ctypes.byref(r),
                                 N.ptr(K), K.stride(0), ctypes.byref(tm), N.ptr(a), N.ptr(b), d,
                                 GRAM_MODES[gram], ctypes.byref(used)), "svmd_train_q")
    return SMOResult.from_struct(r), {"gram_ms": tm.gram_ms, "smo_ms": tm.smo_ms, "total_ms": tm.total_ms,
                                      "gram_alloc_ms": alloc_ms, "kcache": "full", "gram_path": "int8-exact" if used.value else "fp64"}


# ---- the byte path of SVC.fit for uint8 pixel rows: no FP64 copy of the training rows at all
def upload_u8(X: np.ndarray, device) -> torch.Tensor:
    """Host uint8 pixel rows (n, d) -> the same bytes on the device (n, d) uint8."""
    X = np.ascontiguousarray(X, dtype=np.uint8)
    out = device_empty(X.shape, torch.uint8, device)
    ctx = DeviceContext.get(out.device)
    N.check(ctx.lib.svmd_memcpy_h2d(ctx.bind(), N.ptr(out), N.ptr(X), X.nbytes), "svmd_memcpy_h2d")
    return out


def minmax_u8(Xu: torch.Tensor, out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Column min / max (FP64) of device uint8 rows: equal to those of the widened FP64 rows.  With
    ``out`` (2d float64) they are its two halves, so one read-back fetches both."""
    n, d = Xu.shape
    if out is None:
        out = torch.empty(2 * d, dtype=torch.float64, device=Xu.device)
    mn, mx = out[:d], out[d:]
    ctx = _ctx_for(Xu)
    N.check(ctx.lib.svmd_minmax_u8(ctx.bind(), N.ptr(Xu), n, d, N.ptr(mn), N.ptr(mx)), "svmd_minmax_u8")
    return mn, mx


def train_u8(Xu: torch.Tensor, y: torch.Tensor, alpha: torch.Tensor, params: SVMParams, mn: torch.Tensor,
             mx: torch.Tensor, warm: bool = False) -> Optional[Tuple[SMOResult, dict]]:
    """Exact-integer Gram quantised straight from the bytes + SMO (svmd_train_u8): the same Gram,
    trajectory and result as ``train`` on the scaled FP64 rows.  None when the integer plan does not
    apply (the caller takes the FP64-row path)."""
    import time as _t

    n, d = Xu.shape
    ctx = _ctx_for(Xu)
    a, b, _ = _host_stats(mn, mx)  # numpy statistics pass through without a device round trip
    ta = _t.perf_counter()
    K = gram_buffer(n, Xu.device)
    alloc_ms = (_t.perf_counter() - ta) * 1e3
    r, tm, used = N.SvmResult(), N.SvmdTiming(), ctypes.c_int32(0)
    p = params.to_struct()
    N.check(ctx.lib.svmd_train_u8(ctx.bind(), N.ptr(Xu), n, d, N.ptr(a), N.ptr(b), N.ptr(y), N.ptr(alpha), int(warm),
                                  ctypes.byref(p), ctypes.byref(r), N.ptr(K), K.stride(0), ctypes.byref(tm),
                                  ctypes.byref(used)), "svmd_train_u8")
    if not used.value:
        return None
    return SMOResult.from_struct(r), {"gram_ms": tm.gram_ms, "smo_ms": tm.smo_ms, "total_ms": tm.total_ms,
                                      "gram_alloc_ms": alloc_ms, "kcache": "full", "gram_path": "int8-exact",
                                      "rows": "uint8"}


def train_decomp(X: torch.Tensor, y: torch.Tensor, alpha: torch.Tensor, params: SVMParams, mn, mx,
                 working_set: int = 1024, warm: bool = False,
                 trace: Optional["N.DecompTrace"] = None) -> Optional[Tuple[SMOResult, dict]]:
    """Working-set decomposition SMO (svmd_train_decomp, decomp.hip): the reference's stop test on all
    n points, reached by SMO on working sets of up to ``working_set`` points; no n x n Gram.  X: device
    uint8 pixel rows (n, d), or min-max scaled FP64 rows (n, ld) with ``d`` columns (the reference's host
    format, d = len(mn); they quantise into the same integers, so trajectory and model are the uint8 path's).
    warm: alpha holds the start (f = K (alpha y) - y over its nonzero entries).  trace: an
    ``N.DecompTrace`` filled per outer iteration (tests).  FP64 rows without an exact-integer plan
    (real-valued data) are solved with FP64-MFMA kernel values (``gram_path`` "fp64"); uint8 rows
    without one return None (the caller widens them)."""
    u8 = X.dtype == torch.uint8
    if not u8:
        _check_rows(X)
    n, ld = X.shape
    ctx = _ctx_for(X)
    a, b, dd = _host_stats(mn, mx)
    d = ld if u8 else dd
    r, tm, used = N.SvmResult(), N.SvmdTiming(), ctypes.c_int32(0)
    st = (ctypes.c_int64 * 16)()
    p = params.to_struct()
    N.check(ctx.lib.svmd_train_decomp(ctx.bind(), N.ptr(X), int(u8), n, ld, d, N.ptr(a), N.ptr(b), N.ptr(y),
                                      N.ptr(alpha), ctypes.byref(p), int(working_set), int(warm), ctypes.byref(r),
                                      ctypes.byref(tm), st, ctypes.byref(used),
                                      ctypes.byref(trace.struct) if trace is not None else None), "svmd_train_decomp")
    if not used.value:
        return None
    return SMOResult.from_struct(r), {"gram_ms": tm.gram_ms, "smo_ms": tm.smo_ms, "total_ms": tm.total_ms,
                                      "kcache": "none", "gram_path": "fp64" if st[6] else "int8-exact",
                                      "rows": "uint8" if u8 else "fp64", "solver": "decomp", "warm_start": bool(warm),
                                      "warm_columns": int(st[7]), "outer_iterations": int(st[0]),
                                      "inner_iterations": int(st[1]), "working_set": int(st[2]),
                                      "update_columns": int(st[4]), "inner_threads": int(st[5]),
                                      **N.shrink_stats(st)}


def train_decomp_u8(Xu: torch.Tensor, y: torch.Tensor, alpha: torch.Tensor, params: SVMParams, mn, mx,
                    working_set: int = 1024, warm: bool = False) -> Optional[Tuple[SMOResult, dict]]:
    """``train_decomp`` from device uint8 pixel rows."""
    return train_decomp(Xu, y, alpha, params, mn, mx, working_set, warm)


def train_decomp_rows(X: torch.Tensor, y: torch.Tensor, alpha: torch.Tensor, params: SVMParams, mn, mx,
                      working_set: int = 1024, warm: bool = False) -> Optional[Tuple[SMOResult, dict]]:
    """``train_decomp`` from min-max scaled FP64 rows on the device (the reference's host row format)."""
    return train_decomp(X, y, alpha, params, mn, mx, working_set, warm)


def decomp_gemv_u8(Xu: torch.Tensor, mn, mx, gamma: float, cols: np.ndarray, coef: np.ndarray, lo: int = 0,
                   nloc: Optional[int] = None) -> Optional[np.ndarray]:
    """The decomposition solver's f-update GEMV alone (svmd_decomp_gemv_u8): sum_k coef[k] K(i, cols[k])
    for rows i in [lo, lo + nloc) of the exact-integer kernel, in the solver's summation order.  None
    when no exact-integer plan applies."""
    n, d = Xu.shape
    nloc = n - lo if nloc is None else int(nloc)
    cols = np.ascontiguousarray(cols, dtype=np.int32)
    coef = np.ascontiguousarray(coef, dtype=np.float64)
    out = np.empty(nloc, dtype=np.float64)
    a, b, _ = _host_stats(mn, mx)
    used = ctypes.c_int32(0)
    ctx = _ctx_for(Xu)
    N.check(ctx.lib.svmd_decomp_gemv_u8(ctx.bind(), N.ptr(Xu), n, d, N.ptr(a), N.ptr(b), float(gamma), int(lo), nloc,
                                        N.ptr(cols), N.ptr(coef), int(cols.size), N.ptr(out), ctypes.byref(used)),
            "svmd_decomp_gemv_u8")
    return out if used.value else None


def decomp_newton_probe(Kw: np.ndarray, y: np.ndarray, a: np.ndarray, f: np.ndarray, C: float = 10.0,
                        eps: float = 1e-12, max_free: int = 1024, reps: int = 1, device="cuda:0"):
    """One Newton polish step (decomp_newton.h) on the device for a host working set: returns (alpha, f,
    code, phase stamps (100 MHz ticks: free set, K_FF, factorisation, back substitution, step, f; then
    |F|), mean ms per step)."""
    Kw = np.ascontiguousarray(Kw, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.int32)
    a = np.array(a, dtype=np.float64)
    f = np.array(f, dtype=np.float64)
    prof = np.zeros(16, dtype=np.int64)
    code, ms = ctypes.c_int32(0), ctypes.c_double(0.0)
    ctx = _ctx_for(torch.empty(1, device=device))
    N.check(ctx.lib.svmd_decomp_newton_probe(ctx.bind(), N.ptr(Kw), N.ptr(y), len(y), N.ptr(a), N.ptr(f), float(C),
                                             float(eps), int(max_free), int(reps), ctypes.byref(code), N.ptr(prof),
                                             ctypes.byref(ms)), "svmd_decomp_newton_probe")
    return a, f, int(code.value), prof, float(ms.value)


def rbf_gram_u8(Xu: torch.Tensor, gamma: float, mn, mx, out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Exact-integer RBF Gram straight from device uint8 rows (equal to ``rbf_gram_sym`` on the scaled
    FP64 rows); None when the integer plan does not apply."""
    n, d = Xu.shape
    if out is None:
        out = device_empty((n, (n + 1) // 2 * 2), torch.float64, Xu.device)
    a, b, _ = _host_stats(mn, mx)
    used = ctypes.c_int32(0)
    ctx = _ctx_for(Xu)
    N.check(ctx.lib.svmd_rbf_gram_u8(ctx.bind(), N.ptr(Xu), n, d, N.ptr(a), N.ptr(b), float(gamma), N.ptr(out),
                                     out.stride(0), ctypes.byref(used)), "svmd_rbf_gram_u8")
    return out if used.value else None


def sv_rows_u8(Xu: torch.Tensor, idx: torch.Tensor, mn: torch.Tensor, mx: torch.Tensor,
               ld: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Scaled FP64 rows idx (zero padded to ld) and their squared norms from device uint8 rows."""
    d = Xu.shape[1]
    ld = padded_dim(d) if ld is None else ld
    idx = idx.to(torch.int64).contiguous()
    k = idx.numel()
    out = torch.empty((k, ld), dtype=torch.float64, device=Xu.device)
    sqn = torch.empty(k, dtype=torch.float64, device=Xu.device)
    ctx = _ctx_for(Xu)
    N.check(ctx.lib.svmd_sv_rows_u8(ctx.bind(), N.ptr(Xu), d, N.ptr(idx) if k else None, k, N.ptr(mn), N.ptr(mx),
                                    N.ptr(out), ld, N.ptr(sqn)), "svmd_sv_rows_u8")
    return out, sqn


def rbf_gram_sym(X: torch.Tensor, sqn: Optional[torch.Tensor], gamma: float, mn=None, mx=None,
                 gram: str = "auto", out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, str]:
    """Symmetric RBF Gram of preprocessed rows with the svmd_train_q path selection.
    Returns (K, path) with path "int8-exact" or "fp64"."""
    _check_rows(X)
    n = X.shape[0]
    if out is None:
        out = device_empty((n, (n + 1) // 2 * 2), torch.float64, X.device)
    ctx = _ctx_for(X)
    a, b, d = _host_stats(mn, mx)
    used = ctypes.c_int32(0)
    N.check(ctx.lib.svmd_rbf_gram_q(ctx.bind(), N.ptr(X), N.ptr(sqn) if sqn is not None else None, n, X.shape[1],
                                    X.shape[1], N.ptr(a), N.ptr(b), d, float(gamma), N.ptr(out), out.stride(0),
                                    GRAM_MODES[gram], ctypes.byref(used)), "svmd_rbf_gram_q")
    return out, ("int8-exact" if used.value else "fp64")


def decision(Xs: torch.Tensor, ns: torch.Tensor, coef: torch.Tensor, Xq: torch.Tensor, nq: torch.Tensor,
             gamma: float, b: float) -> torch.Tensor:
    """out[i] = sum_k coef[k] K(Xq_i, Xs_k) - b (MFMA cross-kernel + deterministic GEMV)."""
    _check_rows(Xq, "Xq")
    m = Xq.shape[0]
    out = torch.empty(m, dtype=torch.float64, device=Xq.device)
    nsv = Xs.shape[0]
    ctx = _ctx_for(Xq)
    N.check(ctx.lib.svmd_decision(ctx.bind(), N.ptr(Xs) if nsv else None, N.ptr(ns) if nsv else None,
                                  N.ptr(coef) if nsv else None, nsv, Xq.shape[1], N.ptr(Xq), N.ptr(nq), m,
                                  Xq.shape[1], Xq.shape[1], float(gamma), float(b), N.ptr(out)), "svmd_decision")
    return out


def decision_int(X: torch.Tensor, d: int, mn: torch.Tensor, mx: torch.Tensor, coef: torch.Tensor, gamma: float):
    """out[i] = sum_{k < nz} coef[k] K(X_i, X_k), nz = len(coef), on the exact-integer path (the
    Gram's own kernel values) for scaled pixel rows X; None when the rows are not integer pixels."""
    _check_rows(X, "X")
    coef = coef.contiguous()
    k, nz = X.shape[0], coef.numel()
    out = torch.empty(k, dtype=torch.float64, device=X.device)
    used = ctypes.c_int32(0)
    mn_h = np.ascontiguousarray(mn.detach().cpu().numpy(), dtype=np.float64)
    mx_h = np.ascontiguousarray(mx.detach().cpu().numpy(), dtype=np.float64)
    ctx = _ctx_for(X)
    N.check(ctx.lib.svmd_decision_int(ctx.bind(), N.ptr(X), k, X.shape[1], int(d), N.ptr(mn_h), N.ptr(mx_h),
                                      N.ptr(coef), nz, float(gamma), N.ptr(out), ctypes.byref(used)),
            "svmd_decision_int")
    return out if used.value else None


def count_correct(dec: torch.Tensor, y, zero_is_positive: bool = False) -> int:
    """#{i : sign(dec[i]) == y[i]} counted on the device (the reference's predict flag + reduce_sum,
    gpu_svm_main3.cu:277-315); s >= 0 -> +1 if zero_is_positive (cascade rule) else s > 0 -> +1."""
    dec = dec.contiguous()
    m = dec.numel()
    yd = torch.as_tensor(np.ascontiguousarray(y, dtype=np.int32) if not torch.is_tensor(y) else y)
    yd = yd.to(device=dec.device, dtype=torch.int32).contiguous()
    if yd.numel() != m:
        raise ValueError(f"count_correct: {m} decision values but {yd.numel()} labels")
    out = ctypes.c_int64(0)
    if m:
        ctx = _ctx_for(dec)
        N.check(ctx.lib.svmd_count_correct(ctx.bind(), N.ptr(dec), N.ptr(yd), m, int(bool(zero_is_positive)),
                                           ctypes.byref(out)), "svmd_count_correct")
    return int(out.value)


def gather_rows(src: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """dst[k] = src[idx[k]] (device row gather, idx int64 on the same device)."""
    _check_rows(src, "src")
    idx = idx.to(device=src.device, dtype=torch.int64).contiguous()
    out = torch.empty((idx.numel(), src.shape[1]), dtype=torch.float64, device=src.device)
    if idx.numel():
        ctx = _ctx_for(src)
        N.check(ctx.lib.svmd_gather_rows(ctx.bind(), N.ptr(src), src.shape[1], N.ptr(idx), idx.numel(),
                                         N.ptr(out)), "svmd_gather_rows")
    return out
