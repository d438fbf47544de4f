"""Kernel SVM estimator (RBF, one-vs-rest binary) with a CPU oracle backend and an MI355X backend.

``SVC.fit`` runs the reference pipeline — min-max scaling fitted on the training rows
(main3.cpp:57-89), first-order SMO with the reference stop rules (main3.cpp:162-294) — and keeps
the support vectors (alpha > sv_tol, main3.cpp:297-304).  ``predict`` is sign(sum alpha y K - b)
over the SVs (main3.cpp:391-402; the serial/GPU programs map 0 to -1, the cascades to +1 — see
``zero_is_positive``).

Backends
  device="cpu"   native C++ oracle (bit-exact reference arithmetic), ``n_threads`` workers
  device="cuda"  gfx950 kernels: H2D, fused min/max + scale + row norms, the exact-integer int8-MFMA
                 RBF Gram (f64-MFMA for real-valued data) kept resident in HBM, the persistent
                 device SMO (one launch, register-resident slices), MFMA decision function over the
                 SVs; ``kcache="rows"`` (automatic when the Gram does not fit) solves on the HBM row
                 cache instead
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path
from typing import Optional

import numpy as np

from ..utils.config import SVMParams, default_threads
from ..utils.data import MinMaxScaler, check_finite_bounds, check_warm_start


def _resolve_device(device: str) -> str:
    if device == "auto":
        import torch

        return "cuda" if torch.cuda.is_available() else "cpu"
    return device


def _is_u8(X) -> bool:
    return isinstance(X, np.ndarray) and X.dtype == np.uint8


class SVC:
    def __init__(self, C: float = 10.0, gamma: float = 0.00125, tol: float = 1e-5, eps: float = 1e-12,
                 sv_tol: float = 1e-8, max_iter: int = 100000, device: str = "auto", n_threads: int = 0,
                 scale: bool = True, zero_is_positive: bool = False, gram: str = "auto", kcache: str = "auto",
                 wss: str = "first", solver: str = "auto", working_set: int = 1024, shrinking=False):
        if wss not in ("first", "second"):
            raise ValueError("wss must be 'first' (the reference's selection) or 'second'")
        if solver not in ("auto", "smo", "decomp"):
            raise ValueError("solver must be 'auto' (decomp on GPUs, smo on the CPU), 'decomp' (working-set "
                             "decomposition) or 'smo' (the reference's pairwise SMO over all n points)")
        self.params = SVMParams(C=C, gamma=gamma, tau=tol, eps=eps, sv_tol=sv_tol, max_iter=max_iter,
                                n_threads=n_threads if n_threads > 0 else default_threads(),
                                wss=2 if wss == "second" else 1, shrinking=shrinking)
        self.device = device
        self.scale = scale
        self.zero_is_positive = zero_is_positive
        self._sv_host = None
        self.gram = gram  # "auto" | "fp64" | "int" (device backend Gram path, see ops.device.train)
        self.kcache = kcache  # "auto" | "full" (resident Gram) | "rows" (on-demand HBM row cache)
        self._dev = None  # device-side model state (torch tensors)
        # "decomp" (the GPU default): working sets of up to `working_set` points solved in one workgroup
        # with the reference's stop test on all n points (decomp.hip; exact-integer kernel values for
        # pixel rows, FP64 MFMA for real-valued rows; cold or warm start) -- the same support vectors,
        # b within the stop tolerance, a different pair sequence.  "smo": the reference's solver (one
        # pair per iteration over all n points, resident Gram or row cache; the CPU oracle's, the CPU
        # default).  "auto" resolves per fit by device.  shrinking (the decomposition solver, as LIBSVM's /
        # scikit-learn's option): selection and the f update on the active points only, the stop test
        # still on all n (decomp_shrink.h); True, False (the default: measured slower on the headline shapes,
        # profiles/shrinking.md), or a pass every k outer iterations.
        self.solver = solver
        self.working_set = int(working_set)

    # ------------------------------------------------------------------ fit
    def fit(self, X: np.ndarray, y: np.ndarray, alpha0: Optional[np.ndarray] = None) -> "SVC":
        dev = _resolve_device(self.device)
        # uint8 pixel rows stay compact up to the device (8x less H2D; widened to FP64 there)
        X = np.ascontiguousarray(X, dtype=np.uint8 if (dev != "cpu" and _is_u8(X)) else np.float64)
        y = np.ascontiguousarray(y, dtype=np.int32)
        if X.ndim != 2 or y.shape != (X.shape[0],):
            raise ValueError("X must be (n, d) and y (n,)")
        if not np.all(np.abs(y) == 1):
            raise ValueError("labels must be +1/-1 (use svm355.utils.data.one_vs_rest)")
        if alpha0 is not None:
            alpha0 = check_warm_start(alpha0, y, self.params.C)
        t0 = time.perf_counter()
        if dev == "cpu":
            self._fit_cpu(X, y, alpha0)
        else:
            self._fit_cuda(X, y, alpha0, dev)
        self.fit_time_ = time.perf_counter() - t0
        return self

    def _finish(self, alpha: np.ndarray, y: np.ndarray, res) -> None:
        self.alpha_ = alpha
        self.support_ = np.flatnonzero(alpha > self.params.sv_tol).astype(np.int64)
        self.dual_coef_ = alpha[self.support_] * y[self.support_]
        self.support_labels_ = y[self.support_].astype(np.int32)
        self.b_ = res.b
        self.intercept_ = -res.b
        self.n_iter_ = res.iterations
        self.stop_reason_ = res.stop_reason
        self.result_ = res

    def _fit_cpu(self, X, y, alpha0):
        from ..ops import cpu as C

        if self.solver == "decomp":
            raise ValueError("solver='decomp' runs on the GPU (device='cuda'); the CPU oracle is the pairwise SMO")
        if self.scale:
            self.scaler_ = MinMaxScaler().fit(X)
            check_finite_bounds(self.scaler_.min_, self.scaler_.max_)
            Xs = self.scaler_.transform(X)
        else:
            if not np.all(np.isfinite(X)):
                raise ValueError("X holds NaN or infinite values")
            self.scaler_ = None
            Xs = X
        alpha, res, _ = C.smo_train(Xs, y, self.params, alpha=alpha0, warm=alpha0 is not None)
        self._finish(alpha, y, res)
        self.support_vectors_ = Xs[self.support_].copy()
        self.timings_ = {"smo_ms": res.seconds * 1e3}

    def _fit_cuda(self, X, y, alpha0, dev):
        import torch

        from ..ops import device as D

        device = torch.device(dev)
        # auto: the decomposition unless a pairwise-only knob was asked for (second-order pair
        # selection, a forced Gram path or the row cache)
        decomp = self.solver == "decomp" or (self.solver == "auto" and self.params.wss != 2 and self.gram == "auto"
                                             and self.kcache == "auto")
        if decomp:
            if not self.scale:
                if self.solver == "decomp":
                    raise ValueError("solver='decomp' needs scale=True (min-max scaled rows: its exact-integer "
                                     "plan, or the FP64 rows it solves on)")
                decomp = False  # auto without scaling: the pairwise solver
            elif X.dtype == np.uint8 and self._fit_cuda_u8(X, y, alpha0, device, decomp=True):
                return
            # FP64 host rows (the reference's format): scaled on the device, then quantised into the
            # same integers as the byte path (the same trajectory and model), or -- real-valued data --
            # solved on the FP64 rows with FP64-MFMA kernel values
        if (not decomp and X.dtype == np.uint8 and self.scale and self.gram in ("auto", "int")
                and self.kcache in ("auto", "full")
                and os.environ.get("SVM355_U8_TRAIN", "1") != "0" and self._fit_cuda_u8(X, y, alpha0, device)):
            return
        t0 = time.perf_counter()
        Xd = D.upload_rows(X, device)
        yd = torch.from_numpy(y).to(device)
        d = X.shape[1]
        if self.scale:
            mn, mx, sqn = D.minmax_scale_(Xd, d)
            mm_h = mn.as_strided((2 * d,), (1,)).cpu().numpy()  # both bounds (one buffer), one copy
            check_finite_bounds(mm_h[:d], mm_h[d:])
        else:
            mn = mx = None
            sqn = D.row_norms(Xd, d)
            if not np.all(np.isfinite(sqn.cpu().numpy())):  # a NaN / inf anywhere makes its row's norm one
                raise ValueError("X holds NaN or infinite values")
        if alpha0 is not None:
            alpha = torch.from_numpy(np.ascontiguousarray(alpha0, dtype=np.float64)).to(device)
        else:
            alpha = torch.empty(X.shape[0], dtype=torch.float64, device=device)  # the cold start zeroes it
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        out = None
        if decomp:
            out = D.train_decomp_rows(Xd, yd, alpha, self.params, mm_h[:d], mm_h[d:], working_set=self.working_set,
                                      warm=alpha0 is not None)
            if out is None and self.solver == "decomp":
                raise ValueError("solver='decomp': the device rows' stride is not a multiple of 16, n is beyond the "
                                 "solver's 2^31 - 1 rows, or the FP64-row solve's workspace (n x 1024 doubles) does "
                                 "not fit the device")
        if out is not None:
            res, tm = out
        else:  # the pairwise solver (also solver="auto" when the decomposition's workspace does not fit)
            res, tm = D.train(Xd, sqn, yd, alpha, self.params, warm=alpha0 is not None, mn=mn, mx=mx, gram=self.gram,
                              kcache=self.kcache)
        a = alpha.cpu().numpy()
        self._finish(a, y, res)
        idx = torch.from_numpy(self.support_).to(device)
        self._dev = {
            "Xs": D.gather_rows(Xd, idx),
            "ns": sqn[idx].contiguous(),
            "coef": torch.from_numpy(self.dual_coef_).to(device),
            "mn": mn,
            "mx": mx,
            "d": d,
            "device": device,
        }
        if self.scale:
            self.scaler_ = MinMaxScaler(mm_h[:d].copy(), mm_h[d:].copy())
        else:
            self.scaler_ = None
        self._sv_host = None  # scaled SV rows stay on the device; copied to the host on first access
        self.timings_ = {"upload_preprocess_ms": (t1 - t0) * 1e3, **tm}

    def _fit_cuda_u8(self, X, y, alpha0, device, decomp: bool = False) -> bool:
        """uint8 pixel rows, resident Gram: the rows stay bytes on the device -- min/max, the exact-integer
        quantisation and the Gram read them directly, and only the support vectors are ever widened
        to scaled FP64 (for prediction).  Same Gram, trajectory and model as the FP64-row path, minus
        its widen / scale / FP64-quantise passes.  False (nothing fitted) when it does not apply."""
        import torch

        from ..ops import device as D

        n, d = X.shape
        if not decomp and self.kcache == "auto" and not D.gram_fits(n, device):
            return False
        # No PyTorch kernel runs on this path (copies and the library's own kernels only): a process's
        # first PyTorch kernel loads PyTorch's code objects, ~95 ms of a cold first fit
        # (profiles/r3_cold_fit_probe.txt).
        t0 = time.perf_counter()
        Xu = D.upload_u8(X, device)
        yd = torch.from_numpy(y).to(device)
        mmd = torch.empty(2 * d, dtype=torch.float64, device=device)
        mn, mx = D.minmax_u8(Xu, out=mmd)
        if alpha0 is not None:
            alpha = torch.from_numpy(np.ascontiguousarray(alpha0, dtype=np.float64)).to(device)
        else:
            alpha = torch.empty(n, dtype=torch.float64, device=device)  # the cold start zeroes it
        mm = mmd.cpu().numpy()  # one D2H (synchronises) for the plan and the scaler
        mn_h, mx_h = mm[:d].copy(), mm[d:].copy()
        t1 = time.perf_counter()
        if decomp:
            out = D.train_decomp_u8(Xu, yd, alpha, self.params, mn_h, mx_h, working_set=self.working_set,
                                    warm=alpha0 is not None)
        else:
            out = D.train_u8(Xu, yd, alpha, self.params, mn_h, mx_h, warm=alpha0 is not None)
        if out is None:  # nothing ran (not an integer plan): the FP64-row path takes over
            return False
        res, tm = out
        self._finish(alpha.cpu().numpy(), y, res)
        idx = torch.from_numpy(self.support_).to(device)
        Xs, ns = D.sv_rows_u8(Xu, idx, mn, mx)
        self._dev = {"Xs": Xs, "ns": ns, "coef": torch.from_numpy(self.dual_coef_).to(device), "mn": mn, "mx": mx,
                     "d": d, "device": device}
        self.scaler_ = MinMaxScaler(mn_h, mx_h)
        self._sv_host = None
        self.timings_ = {"upload_preprocess_ms": (t1 - t0) * 1e3, **tm}
        return True

    @property
    def support_vectors_(self) -> np.ndarray:
        """Scaled support-vector rows (host copy, fetched lazily from the device model)."""
        if self._sv_host is None and self._dev is not None:
            self._sv_host = self._dev["Xs"][:, : self._dev["d"]].cpu().numpy()
        return self._sv_host

    @support_vectors_.setter
    def support_vectors_(self, value) -> None:
        self._sv_host = value

    # ------------------------------------------------------------------ inference
    def _n_features(self) -> Optional[int]:
        if self._dev is not None:
            return int(self._dev["d"])
        if self.scaler_ is not None and self.scaler_.min_ is not None:
            return int(np.size(self.scaler_.min_))
        sv = self.support_vectors_
        return int(sv.shape[1]) if sv is not None and np.ndim(sv) == 2 else None

    def _check_X(self, X) -> None:
        d = self._n_features()
        if np.ndim(X) != 2 or (d is not None and np.shape(X)[1] != d):
            raise ValueError(f"X must be (m, {d}) like the training rows, got shape {np.shape(X)}")

    def decision_function(self, X: np.ndarray) -> np.ndarray:
        self._check_X(X)
        if self._dev is not None:
            return self._device_decision(X).cpu().numpy()
        return self._host_decision(X)

    def _device_decision(self, X: np.ndarray):
        """Decision values as a device tensor (device models only)."""
        from ..ops import device as D

        X = np.ascontiguousarray(X, dtype=np.uint8 if _is_u8(X) else np.float64)
        dv = self._dev
        Xq = D.upload_rows(X, dv["device"])
        if self.scale:
            _, _, nq = D.minmax_scale_(Xq, dv["d"], dv["mn"], dv["mx"])
        else:
            nq = D.row_norms(Xq, dv["d"])
        return D.decision(dv["Xs"], dv["ns"], dv["coef"], Xq, nq, self.params.gamma, self.b_)

    def _host_decision(self, X: np.ndarray) -> np.ndarray:
        from ..ops import cpu as C

        X = np.ascontiguousarray(X, dtype=np.float64)
        Xq = self.scaler_.transform(X) if self.scaler_ is not None else X
        return C.decision(self.support_vectors_, self.support_labels_, self.alpha_[self.support_], Xq,
                          self.params.gamma, self.b_, self.params.n_threads)

    def predict(self, X: np.ndarray) -> np.ndarray:
        dec = self.decision_function(X)
        pos = dec >= 0 if self.zero_is_positive else dec > 0
        return np.where(pos, 1, -1).astype(np.int32)

    def score(self, X: np.ndarray, y: np.ndarray) -> float:
        """Accuracy.  Device models count the correct signs on the device (count_correct)."""
        y = np.asarray(y)
        if self._dev is not None and len(y):
            from ..ops import device as D

            self._check_X(X)
            return D.count_correct(self._device_decision(X), y, self.zero_is_positive) / len(y)
        return float(np.mean(self.predict(X) == y))

    # ------------------------------------------------------------------ persistence
    def save(self, directory: str | os.PathLike, ids: Optional[np.ndarray] = None) -> None:
        """Reference model files (final_sv_{ids,labels,alphas}.txt, final_b.txt) + loadable extras."""
        from ..models.model_io import save_model

        save_model(directory, ids=self.support_ if ids is None else ids, labels=self.support_labels_,
                   alphas=self.alpha_[self.support_], b=self.b_, sv_rows=self.support_vectors_,
                   scaler=self.scaler_, params=self.params, meta={"n_iter": self.n_iter_,
                                                                  "stop_reason": self.stop_reason_})

    @classmethod
    def load(cls, directory: str | os.PathLike, device: str = "cpu") -> "SVC":
        from ..models.model_io import load_model

        m = load_model(directory)
        p = m["params"]
        svc = cls(C=p.C, gamma=p.gamma, tol=p.tau, eps=p.eps, sv_tol=p.sv_tol, max_iter=p.max_iter, device=device,
                  scale=m["scaler"] is not None)
        svc.scaler_ = m["scaler"]
        svc.support_ = m["ids"]
        svc.support_labels_ = m["labels"]
        svc.b_ = m["b"]
        svc.intercept_ = -m["b"]
        svc.support_vectors_ = m["sv_rows"]
        alphas = m["alphas"]
        # alpha_ is indexed by training row; a loaded model only knows its SVs.
        svc.alpha_ = np.zeros(int(svc.support_.max()) + 1 if len(svc.support_) else 0)
        svc.alpha_[svc.support_] = alphas
        svc.dual_coef_ = alphas * svc.support_labels_
        if _resolve_device(device) != "cpu":
            svc._upload_model(_resolve_device(device))
        return svc

    def _device_model_from_u8(self, X_sv: np.ndarray, dev: str) -> None:
        """The device model of a fit whose rows are uint8 pixels and whose alphas, b and scaler are set
        (the distributed trainers): only the SV rows' bytes cross PCIe, widened and scaled on the device
        (svmd_sv_rows_u8) -- no host FP64 transform and no FP64 upload (~1 MB instead of 8.6 MB at 60k).
        No PyTorch kernel runs (copies and the library's own kernels only)."""
        import torch

        from ..ops import device as D

        device = torch.device(dev)
        X_sv = np.ascontiguousarray(X_sv, dtype=np.uint8)
        k, d = X_sv.shape
        mm = torch.from_numpy(np.concatenate([self.scaler_.min_, self.scaler_.max_]).astype(np.float64)).to(device)
        mn, mx = mm[:d], mm[d:]
        if k:
            Xu = D.upload_u8(X_sv, device)
            idx = torch.from_numpy(np.arange(k, dtype=np.int64)).to(device)
            Xs, ns = D.sv_rows_u8(Xu, idx, mn, mx)
        else:
            Xs = torch.empty((0, D.padded_dim(d)), dtype=torch.float64, device=device)
            ns = torch.empty(0, dtype=torch.float64, device=device)
        self._dev = {"Xs": Xs, "ns": ns, "coef": torch.from_numpy(np.ascontiguousarray(self.dual_coef_)).to(device),
                     "mn": mn, "mx": mx, "d": d, "device": device}
        self._sv_host = None

    def _upload_model(self, dev: str) -> None:
        import torch

        from ..ops import device as D

        device = torch.device(dev)
        d = self.support_vectors_.shape[1]
        Xs = D.upload_rows(self.support_vectors_, device)
        self._dev = {
            "Xs": Xs,
            "ns": D.row_norms(Xs, d),
            "coef": torch.from_numpy(np.ascontiguousarray(self.dual_coef_)).to(device),
            "mn": torch.from_numpy(self.scaler_.min_).to(device) if self.scaler_ is not None else None,
            "mx": torch.from_numpy(self.scaler_.max_).to(device) if self.scaler_ is not None else None,
            "d": d,
            "device": device,
        }
