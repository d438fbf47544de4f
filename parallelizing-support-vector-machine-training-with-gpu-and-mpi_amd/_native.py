"""ctypes bindings to the native runtime (``lib/libsvm355_core.so`` and ``lib/libsvm355_hip.so``).

The C ABI is declared in ``csrc/include/svm355.h`` and ``csrc/include/svm355_device.h``.  The
libraries are built in-tree by :mod:`svm355.build`; the CPU core is rebuilt on demand when it is
missing (g++ only, a few seconds), the device library must have been built beforehand (hipcc).
Every failing native call raises :class:`NativeError` carrying ``svm_last_error()``; there is no
silent fallback from the device library to anything else.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, c_char_p, c_double, c_int32, c_int64, c_uint64, c_void_p
from pathlib import Path

LIB_DIR = Path(os.environ.get("SVM355_LIB_DIR") or Path(__file__).resolve().parent / "lib")  # override: A/B builds

_lock = threading.Lock()
_core = None
_hip = None

STOP_NAMES = {
    0: "running",
    1: "converged",
    2: "no_candidate",
    3: "infeasible",
    4: "nonpositive_eta",
    5: "max_iter",
}


class NativeError(RuntimeError):
    pass


class SvmParams(ctypes.Structure):
    _fields_ = [
        ("C", c_double),
        ("gamma", c_double),
        ("tau", c_double),
        ("eps", c_double),
        ("sv_tol", c_double),
        ("max_iter", c_int64),
        ("n_threads", c_int32),
        ("verbose", c_int32),
        ("wss", c_int32),
        ("shrink", c_int32),
    ]


class SvmResult(ctypes.Structure):
    _fields_ = [
        ("iterations", c_int64),
        ("b", c_double),
        ("b_high", c_double),
        ("b_low", c_double),
        ("stop_reason", c_int32),
        ("reserved", c_int32),
        ("n_sv", c_int64),
        ("seconds", c_double),
    ]


class SvmdTiming(ctypes.Structure):
    _fields_ = [
        ("h2d_ms", c_double),
        ("preprocess_ms", c_double),
        ("gram_ms", c_double),
        ("smo_ms", c_double),
        ("total_ms", c_double),
    ]


class SvmCascadeCfg(ctypes.Structure):
    _fields_ = [
        ("tree", c_int32),
        ("max_rounds", c_int32),
        ("params", SvmParams),
        ("log", c_int32),
        ("resume", c_int32),
        ("checkpoint_dir", c_char_p),
        ("comm_timeout_s", c_double),
        ("fail_rank", c_int32),
        ("fail_round", c_int32),
        ("fail_stall_s", c_double),
        ("solver", c_int32),
        ("reserved", c_int32),
    ]


class SvmCascadeOut(ctypes.Structure):
    _fields_ = [
        ("world", c_int32),
        ("rank", c_int32),
        ("rounds", c_int32),
        ("converged", c_int32),
        ("b", c_double),
        ("train_ms", c_double),
        ("d", c_int64),
        ("n_sv", c_int64),
        ("ids", POINTER(c_int64)),
        ("y", POINTER(c_int32)),
        ("alpha", POINTER(c_double)),
        ("sv_rows", POINTER(c_double)),
        ("mn", POINTER(c_double)),
        ("mx", POINTER(c_double)),
        ("n_hist", c_int64),
        ("sv_history", POINTER(c_int64)),
        ("round_ms", POINTER(c_double)),
        ("n_merged", c_int64),
        ("merged_history", POINTER(c_int64)),
        ("n_solves", c_int64),
        ("solves", POINTER(c_double)),
        ("n_ranks", c_int64),
        ("rank_train_ms", POINTER(c_double)),
        ("transport", ctypes.c_char * 16),
        ("backend", ctypes.c_char * 16),
        ("phase_ms", c_double * 11),
    ]


class SvmDecompTrace(ctypes.Structure):
    _fields_ = [
        ("cap", c_int64),
        ("count", c_int64),
        ("n", c_int64),
        ("m", c_void_p),
        ("W", c_void_p),
        ("moved", c_void_p),
        ("cols", c_void_p),
        ("coef", c_void_p),
        ("inner", c_void_p),
        ("bounds", c_void_p),
        ("alpha", c_void_p),
        ("f", c_void_p),
    ]


DECOMP_MAX_WS = 1024  # svm355.h SVM_DECOMP_MAX_WS


class DecompTrace:
    """Host buffers of an ``svm_decomp_trace`` (per outer iteration of a decomposition solve: working
    set, moved columns and coefficients, inner iterations, bounds, optionally alpha / f snapshots)."""

    def __init__(self, cap: int, n: int = 0):
        import numpy as np

        w = DECOMP_MAX_WS
        self.m = np.zeros(cap, dtype=np.int32)
        self.W = np.full((cap, w), -1, dtype=np.int32)
        self.moved = np.zeros(cap, dtype=np.int32)
        self.cols = np.full((cap, w), -1, dtype=np.int32)
        self.coef = np.zeros((cap, w), dtype=np.float64)
        self.inner = np.zeros(cap, dtype=np.int64)
        self.bounds = np.zeros((cap, 2), dtype=np.float64)
        self.alpha = np.zeros((cap, n), dtype=np.float64) if n else None
        self.f = np.zeros((cap, n), dtype=np.float64) if n else None
        self.struct = SvmDecompTrace(cap, 0, n, *(ptr(a) for a in (self.m, self.W, self.moved, self.cols, self.coef,
                                                                    self.inner, self.bounds, self.alpha, self.f)))

    @property
    def count(self) -> int:
        return int(self.struct.count)

    def records(self) -> list:
        """One dict per recorded outer iteration (arrays trimmed to their sizes)."""
        out = []
        for o in range(self.count):
            m, k = int(self.m[o]), int(self.moved[o])
            rec = {"m": m, "W": self.W[o, :m].copy(), "moved": k, "cols": self.cols[o, :k].copy(),
                   "coef": self.coef[o, :k].copy(), "inner": int(self.inner[o]), "bounds": self.bounds[o].copy()}
            if self.alpha is not None:
                rec["alpha"] = self.alpha[o].copy()
                rec["f"] = self.f[o].copy()
            out.append(rec)
        return out


SOLVE_COLS = 14  # svm355.h SVM_CASCADE_SOLVE_COLS
CASCADE_PHASES = ("upload", "scale", "bcast", "assemble", "solve", "select", "gather", "sendrecv", "checkpoint",
                  "final", "setup")


_P = c_void_p  # raw pointers are passed as integers / c_void_p
_CORE_SIGS = {
    "svm_last_error": (c_char_p, []),
    "svm_default_params": (None, [POINTER(SvmParams)]),
    "svm_stop_message": (c_char_p, [c_int32]),
    "svm_csv_load": (c_void_p, [c_char_p, c_int64, c_int32, c_int32]),
    "svm_dataset_dims": (c_int32, [c_void_p, POINTER(c_int64), POINTER(c_int64)]),
    "svm_dataset_copy": (c_int32, [c_void_p, _P, _P, _P]),
    "svm_dataset_free": (None, [c_void_p]),
    "svm_csv_write": (c_int32, [c_char_p, _P, _P, c_int64, c_int64]),
    "svm_synth_mnist": (c_int32, [c_uint64, c_int64, c_int64, _P, _P, c_int32]),
    "svm_minmax": (c_int32, [_P, c_int64, c_int64, _P, _P]),
    "svm_scale": (c_int32, [_P, c_int64, c_int64, _P, _P]),
    "svm_rbf": (c_double, [_P, _P, c_int64, c_double]),
    "svm_rbf_matrix": (c_int32, [_P, c_int64, _P, c_int64, c_int64, c_double, _P, c_int32]),
    "svm_smo_train": (c_int32, [_P, _P, c_int64, c_int64, _P, c_int32, POINTER(SvmParams),
                                POINTER(SvmResult), _P, c_int64]),
    "svm_smo_train_gram": (c_int32, [_P, c_int64, _P, c_int64, _P, c_int32, POINTER(SvmParams),
                                     POINTER(SvmResult), _P, c_int64]),
    "svm_decomp_train_gram": (c_int32, [_P, c_int64, _P, c_int64, _P, c_int32, POINTER(SvmParams), c_int32, c_double,
                                        c_int32, POINTER(SvmResult), POINTER(c_int64), POINTER(SvmDecompTrace)]),
    "svm_crash_handler_install": (c_int32, [c_char_p]),
    "svm_decomp_gemv_ref": (c_int32, [_P, c_int64, c_int64, _P, _P, c_int64, _P]),
    "svm_decomp_newton_step": (c_int32, [_P, c_int64, _P, c_int32, _P, _P, c_double, c_double, c_int32, POINTER(c_int32)]),
    "svm_decomp_rank_train_gram": (c_int32, [_P, _P, c_int64, _P, c_int64, _P, c_int32, POINTER(SvmParams), c_int32,
                                             c_double, c_int32, POINTER(SvmResult), POINTER(c_int64)]),
    "svm_decomp_group_train_gram": (c_int32, [c_int32, _P, c_int64, _P, c_int64, _P, c_int32, POINTER(SvmParams),
                                              c_int32, c_double, c_int32, POINTER(SvmResult), POINTER(c_int64),
                                              c_double]),
    "svm_decision": (c_int32, [_P, _P, _P, c_int64, _P, c_int64, c_int64, c_double, c_double, _P,
                               c_int32]),
    "svm_sv_indices": (c_int64, [_P, c_int64, c_double, _P]),
    "svm_model_save": (c_int32, [c_char_p, _P, _P, _P, c_int64, c_double]),
    "svm_cascade_default_cfg": (None, [POINTER(SvmCascadeCfg)]),
    "svm_cascade_fit_cpu": (POINTER(SvmCascadeOut), [_P, _P, c_int64, c_int64, c_int32, POINTER(SvmCascadeCfg)]),
    "svm_cascade_free": (None, [POINTER(SvmCascadeOut)]),
    "svm_cascade_rank_fit_cpu": (POINTER(SvmCascadeOut), [_P, _P, _P, _P, c_int64, c_int64, c_int64,
                                                          POINTER(SvmCascadeCfg)]),
    "svm_loopback_exercise": (c_int32, [c_int32, c_char_p, c_int32, c_double, POINTER(c_double)]),
    "svm_preflight_script": (c_int32, [c_int32, c_int64, c_char_p, c_int64]),
}

_HIP_SIGS = {
    "svmd_padded_dim": (c_int64, [c_int64]),
    "svmd_device_count": (c_int32, [POINTER(c_int32)]),
    "svmd_alloc": (c_void_p, [c_void_p, c_int64]),
    "svmd_free": (None, [c_void_p, c_void_p]),
    "svmd_memcpy_h2d": (c_int32, [c_void_p, _P, _P, c_int64]),
    "svmd_memcpy_d2h": (c_int32, [c_void_p, _P, _P, c_int64]),
    "svmd_create": (c_void_p, [c_int32]),
    "svmd_destroy": (None, [c_void_p]),
    "svmd_set_stream": (c_int32, [c_void_p, c_void_p]),
    "svmd_synchronize": (c_int32, [c_void_p]),
    "svmd_upload_rows": (c_int32, [c_void_p, _P, c_int64, c_int64, _P, c_int64]),
    "svmd_upload_rows_u8": (c_int32, [c_void_p, _P, c_int64, c_int64, _P, c_int64]),
    "svmd_minmax": (c_int32, [c_void_p, _P, c_int64, c_int64, c_int64, _P, _P]),
    "svmd_preprocess":(c_int32, [c_void_p, _P, c_int64, c_int64, c_int64, _P, _P, _P, c_int32]),
    "svmd_row_norms": (c_int32, [c_void_p, _P, c_int64, c_int64, c_int64, _P]),
    "svmd_rbf_gram": (c_int32, [c_void_p, _P, _P, c_int64, c_int64, _P, _P, c_int64, c_int64, c_int64,
                                c_double, _P, c_int64, c_int32]),
    "svmd_smo": (c_int32, [c_void_p, _P, c_int64, _P, c_int64, _P, c_int32, POINTER(SvmParams),
                           POINTER(SvmResult), _P, c_int64]),
    "svmd_release_cache": (c_int32, [c_void_p]),
    "svmd_release_slab": (c_int32, [c_void_p]),
    "svmd_set_ccache_frac": (c_int32, [c_void_p, c_double]),
    "svmd_cache_bytes": (c_int32, [c_void_p, POINTER(c_int64), POINTER(c_int64)]),
    "svmd_selftest_exp": (c_int32, [c_void_p, _P, c_int64, _P, _P]),
    "svmd_smo_multi": (c_int32, [c_void_p, _P, c_int64, _P, c_int64, c_int32, _P, POINTER(SvmParams),
                                 POINTER(SvmResult), POINTER(c_int32)]),
    "svmd_train": (c_int32, [c_void_p, _P, _P, c_int64, c_int64, c_int64, _P, _P, c_int32,
                             POINTER(SvmParams), POINTER(SvmResult), _P, c_int64, POINTER(SvmdTiming)]),
    "svmd_train_q": (c_int32, [c_void_p, _P, _P, c_int64, c_int64, c_int64, _P, _P, c_int32,
                               POINTER(SvmParams), POINTER(SvmResult), _P, c_int64, POINTER(SvmdTiming),
                               _P, _P, c_int64, c_int32, POINTER(c_int32)]),
    "svmd_train_rows": (c_int32, [c_void_p, _P, _P, c_int64, c_int64, c_int64, _P, _P, c_int32, POINTER(SvmParams),
                                  POINTER(SvmResult), _P, _P, c_int32, c_int64, POINTER(c_int32), _P, c_int64]),
    "svmd_rbf_gram_q": (c_int32, [c_void_p, _P, _P, c_int64, c_int64, c_int64, _P, _P, c_int64, c_double, _P,
                                  c_int64, c_int32, POINTER(c_int32)]),
    "svmd_decision": (c_int32, [c_void_p, _P, _P, _P, c_int64, c_int64, _P, _P, c_int64, c_int64, c_int64,
                                c_double, c_double, _P]),
    "svmd_decision_int": (c_int32, [c_void_p, _P, c_int64, c_int64, c_int64, _P, _P, _P, c_int64, c_double, _P,
                                    POINTER(c_int32)]),
    "svmd_gather_rows": (c_int32, [c_void_p, _P, c_int64, _P, c_int64, _P]),
    "svmd_train_u8": (c_int32, [c_void_p, _P, c_int64, c_int64, _P, _P, _P, _P, c_int32, POINTER(SvmParams),
                                POINTER(SvmResult), _P, c_int64, POINTER(SvmdTiming), POINTER(c_int32)]),
    "svmd_train_decomp_u8": (c_int32, [c_void_p, _P, c_int64, c_int64, _P, _P, _P, _P, POINTER(SvmParams), c_int32,
                                       POINTER(SvmResult), POINTER(SvmdTiming), POINTER(c_int64),
                                       POINTER(c_int32)]),
    "svmd_train_decomp_rows": (c_int32, [c_void_p, _P, c_int64, c_int64, c_int64, _P, _P, _P, _P, POINTER(SvmParams),
                                         c_int32, POINTER(SvmResult), POINTER(SvmdTiming), POINTER(c_int64),
                                         POINTER(c_int32)]),
    "svmd_train_decomp": (c_int32, [c_void_p, _P, c_int32, c_int64, c_int64, c_int64, _P, _P, _P, _P,
                                    POINTER(SvmParams), c_int32, c_int32, POINTER(SvmResult), POINTER(SvmdTiming),
                                    POINTER(c_int64), POINTER(c_int32), POINTER(SvmDecompTrace)]),
    "svmd_decomp_newton_probe": (c_int32, [c_void_p, _P, _P, c_int32, _P, _P, c_double, c_double, c_int32, c_int32,
                                            POINTER(c_int32), _P, POINTER(c_double)]),
    "svmd_decomp_gemv_u8": (c_int32, [c_void_p, _P, c_int64, c_int64, _P, _P, c_double, c_int64, c_int64, _P, _P,
                                      c_int32, _P, POINTER(c_int32)]),
    "svmd_minmax_u8": (c_int32, [c_void_p, _P, c_int64, c_int64, _P, _P]),
    "svmd_cascade_group_decomp": (c_int32, [c_void_p, _P, _P, c_int64, c_int64, POINTER(SvmParams), c_int32, _P,
                                            POINTER(SvmResult), POINTER(c_int64), _P, _P]),
    "svmd_cascade_group_decomp_rows": (c_int32, [c_void_p, _P, _P, c_int64, c_int64, POINTER(SvmParams), c_int32,
                                                 _P, POINTER(SvmResult), POINTER(c_int64), _P, _P]),
    "svmd_cascade_rank_decomp": (c_int32, [c_void_p, _P, _P, c_int64, c_int64, POINTER(SvmParams), c_int32, _P,
                                           POINTER(SvmResult), POINTER(c_int64), _P, _P]),
    "svmd_cascade_rank_decomp_rows": (c_int32, [c_void_p, _P, _P, c_int64, c_int64, POINTER(SvmParams), c_int32,
                                                _P, POINTER(SvmResult), POINTER(c_int64), _P, _P]),
    "svmd_rbf_gram_u8": (c_int32, [c_void_p, _P, c_int64, c_int64, _P, _P, c_double, _P, c_int64, POINTER(c_int32)]),
    "svmd_sv_rows_u8": (c_int32, [c_void_p, _P, c_int64, _P, c_int64, _P, _P, _P, c_int64, _P]),
    "svmd_count_correct": (c_int32, [c_void_p, _P, _P, c_int64, c_int32, POINTER(c_int64)]),
    "svmd_cascade_group_create": (c_void_p, [c_int32, c_char_p, c_double]),
    "svmd_cascade_group_world": (c_int32, [c_void_p]),
    "svmd_cascade_group_fit": (POINTER(SvmCascadeOut), [c_void_p, _P, c_int32, _P, c_int64, c_int64,
                                                        POINTER(SvmCascadeCfg)]),
    "svmd_cascade_group_destroy": (None, [c_void_p]),
    "svmd_nccl_unique_id_bytes": (c_int64, []),
    "svmd_nccl_unique_id": (c_int32, [_P, c_int64]),
    "svmd_cascade_rank_create": (c_void_p, [c_int32, _P, c_int32, c_int32, c_double]),
    "svmd_cascade_rank_create_hostcomm": (c_void_p, [_P, c_int32, c_double]),
    "svmd_cascade_group_decomp_solo": (c_int64, [c_void_p, _P, c_int64]),
    "svmd_cascade_group_decomp_waits": (c_int64, [c_void_p, _P, c_int64]),
    "svmd_cascade_rank_decomp_wait": (c_double, [c_void_p]),
    "svmd_cascade_rank_fit": (POINTER(SvmCascadeOut), [c_void_p, _P, c_int32, _P, _P, c_int64, c_int64, c_int64,
                                                       POINTER(SvmCascadeCfg)]),
    "svmd_cascade_rank_barrier": (c_int32, [c_void_p]),
    "svmd_cascade_group_exercise": (c_int32, [c_void_p, c_char_p, c_double]),
    "svmd_cascade_rank_exercise": (c_int32, [c_void_p, c_char_p, c_double]),
    "svmd_cascade_group_broken": (c_int32, [c_void_p]),
    "svmd_rccl_info": (c_int32, [POINTER(c_int32), POINTER(c_int32), c_char_p, c_int64]),
    "svmd_cascade_rank_destroy": (None, [c_void_p]),
    "svmd_dsmo_create": (c_void_p, [c_int32, c_int32, c_double]),
    "svmd_dsmo_destroy": (None, [c_void_p]),
    "svmd_dsmo_world": (c_int32, [c_void_p]),
    "svmd_dsmo_plan": (c_int32, [c_int64, c_int32, c_int32, c_int32, _P]),
    "svmd_dsmo_fit": (c_int32, [c_void_p, _P, c_int32, _P, c_int64, c_int64, POINTER(SvmParams), _P,
                                POINTER(SvmResult), _P, _P, c_int64, _P, _P, _P]),
    "svmd_dsmo_rank_create": (c_void_p, [c_int32, c_int32, c_int32, c_double]),
    "svmd_dsmo_handle_bytes": (c_int64, []),
    "svmd_dsmo_rank_handle": (c_int32, [c_void_p, _P, c_int64]),
    "svmd_dsmo_rank_connect": (c_int32, [c_void_p, _P]),
    "svmd_dsmo_rank_prepare": (c_int32, [c_void_p, _P, c_int32, _P, c_int64, c_int64, POINTER(SvmParams)]),
    "svmd_dsmo_rank_solve": (c_int32, [c_void_p, _P, POINTER(SvmResult), _P, _P, _P, _P, _P]),
    "svmd_trace_push": (None, [c_char_p]),
    "svmd_trace_pop": (None, []),
}


def _bind(lib, sigs):
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def core():
    """The CPU core library (built on demand)."""
    global _core
    if _core is not None:
        return _core
    with _lock:
        if _core is None:
            path = LIB_DIR / "libsvm355_core.so"
            if not path.exists() or os.environ.get("SVM355_REBUILD"):
                from . import build

                build.build_core()
            # RTLD_GLOBAL so the device library resolves the core's symbols from this copy.
            _core = _bind(ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL), _CORE_SIGS)
            crash = os.environ.get("SVM355_CRASH_MAPS")
            if crash:  # crash evidence: signal, PC, backtrace and /proc/self/maps appended to this file
                check(_core.svm_crash_handler_install(crash.replace("{pid}", str(os.getpid())).encode()),
                      "svm_crash_handler_install")
    return _core


def hip():
    """The HIP/gfx950 device library.  Raises if it is missing or cannot be loaded."""
    global _hip
    if _hip is not None:
        return _hip
    core()
    with _lock:
        if _hip is None:
            path = LIB_DIR / "libsvm355_hip.so"
            if not path.exists():
                raise NativeError(
                    f"{path} is missing: build it with `python -m svm355.build` (hipcc, gfx950)")
            try:
                _hip = _bind(ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL), _HIP_SIGS)
            except OSError as e:  # pragma: no cover - depends on the ROCm install
                raise NativeError(f"cannot load {path}: {e}") from e
    return _hip


def last_error() -> str:
    msg = core().svm_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = "native call") -> None:
    if rc != 0:
        raise NativeError(f"{what} failed (status {rc}): {last_error()}")


def ptr(a) -> int:
    """Raw address of a numpy array or torch tensor (contiguity is the caller's contract)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data


def newton_step_probe(Kw, y, a, f, C=10.0, eps=1e-12, max_free=1024):
    """One Newton polish step (decomp_newton.h newton_step_ref) on a working set: Kw (m x m), labels,
    alpha, f by position.  Returns (alpha, f, code: 0 none, 1 full step, 2 cut at a bound)."""
    import numpy as np

    Kw = np.ascontiguousarray(Kw, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.int32)
    a = np.array(a, dtype=np.float64)
    f = np.array(f, dtype=np.float64)
    code = c_int32(0)
    check(core().svm_decomp_newton_step(ptr(Kw), Kw.shape[1], ptr(y), len(y), ptr(a), ptr(f), float(C), float(eps),
                                        int(max_free), code), "svm_decomp_newton_step")
    return a, f, int(code.value)


def shrink_stats(st) -> dict:
    """The decomposition solver's shrinking and Newton-polish counters (stats[8:13] of a solve,
    decomp_shrink.h / decomp_newton.h)."""
    return {"unshrinks": int(st[8]), "shrink_passes": int(st[9]), "min_active": int(st[10]),
            "repacks": int(st[11]), "newton_steps": int(st[12])}


def params_struct(C=10.0, gamma=0.00125, tau=1e-5, eps=1e-12, sv_tol=1e-8, max_iter=100000,
                  n_threads=1, verbose=0, wss=1, shrink=0) -> SvmParams:
    return SvmParams(float(C), float(gamma), float(tau), float(eps), float(sv_tol), int(max_iter),
                     int(n_threads), int(verbose), int(wss), int(shrink))
