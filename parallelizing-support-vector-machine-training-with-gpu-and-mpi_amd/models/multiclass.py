"""Multi-class RBF SVM, one-vs-rest over a SHARED kernel matrix.

The reference trains a single one-vs-rest classifier (digit "1" vs the rest, main3.cpp:49-52).
Training all ten digits the same way is ten SMO solves on the same rows: the RBF Gram does not
depend on the labels, so on the device it is computed once (exact-integer int8 MFMA path for
pixel data), kept resident in HBM and reused by every class's SMO.  The solves are independent and
each is latency-bound on one XCD's worth of workgroups, so they run in ONE launch
(smo.hip smo_multi_kernel): every XCD forms a team of workgroups that exchanges its per-iteration
candidates through that XCD's L2 and pulls classes from a shared queue — eight classes at once, and
a team that finishes early takes the next class.  (``solver="streams"``: one persistent solve per
class on ``concurrent_solves`` streams instead.)  ``solver="decomp"`` (the GPU default, as for ``SVC``):
no Gram at all -- every class is
the working-set decomposition solver of ``SVC(solver="decomp")`` (decomp.hip) on the one copy of the
device rows, the classes on ``concurrent_solves`` host threads of a persistent pool (each with its
device context and stream): the one-workgroup inner solves of different classes run side by side on
different CUs and their f-update GEMVs share the chip.  Prediction evaluates one
cross-kernel block against the union of all classes' support vectors and applies every class's
dual coefficients with one FP64 matrix product; the predicted label is the arg-max decision value.

On the CPU (``device="cpu"``) each class is the native oracle (bit-exact reference arithmetic).

Across GPUs (``fit(..., transport=t)``, one rank per GPU over RCCL): the classes are dealt
round-robin to the ranks, each rank builds the Gram on its own GPU and solves its classes, and one
all-reduce of the (classes x n) alpha matrix plus per-class b/iterations gives every rank the whole
model — the one-vs-rest analogue of the reference's data-parallel cascade, with no cross-rank
dependency inside a solve.
"""
from __future__ import annotations

import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

import numpy as np

from ..utils.config import SVMParams, default_threads
from ..utils.data import MinMaxScaler, check_finite_bounds
from ..utils.trace import trace_range


_POOL_LOCK = threading.Lock()
_POOL: list = [None, 0]  # the one persistent pool of the decomposition class solves, and its width
_TLS = threading.local()


def _release_pool(pool: ThreadPoolExecutor, workers: int, timeout_s: float) -> bool:
    """Every thread of `pool` hands back its device slabs (one task per thread, all held at a barrier so
    that no thread takes two); False when the barrier timed out (a fit was using the pool)."""
    from ..ops import device as D

    barrier = threading.Barrier(workers)

    def release(_):
        try:
            barrier.wait(timeout_s)
        except threading.BrokenBarrierError:
            return False
        D.release_gram_buffers()
        return True

    return all(list(pool.map(release, range(workers))))


def _pool(workers: int) -> ThreadPoolExecutor:
    """The persistent pool for the decomposition class solves: its threads keep their device contexts
    (DeviceContext is per thread), streams and column-cache slabs from one fit to the next.  ONE pool at a
    time: a fit with another width first has the old pool's threads hand back their slabs and
    shuts it down, so the slabs never pile up across widths and the threads stay bounded.  (If the old pool
    is busy -- a concurrent fit of thread ranks -- it is left to finish and dropped; its threads exit with it.)"""
    workers = max(1, int(workers))
    with _POOL_LOCK:
        pool, width = _POOL
        if pool is not None and width == workers:
            return pool
        if pool is not None:
            if _release_pool(pool, width, 2.0):
                pool.shutdown(wait=False)
        _POOL[0] = ThreadPoolExecutor(max_workers=workers, thread_name_prefix=f"svm355-ovr{workers}")
        _POOL[1] = workers
        return _POOL[0]


def release_solver_caches(timeout_s: float = 5.0) -> bool:
    """Hand back the device memory the one-vs-rest decomposition solves keep between fits -- each pool
    thread's column-cache slab (large n; at most half the HBM over the pool), invisible to PyTorch's
    allocator -- on every thread of the pool (``ops.device.release_gram_buffers`` acts on the calling
    thread only).  Call it with no fit running; False when the pool's barrier timed out (a fit was using
    it) and its slabs were kept.  ``ops.device.device_empty`` calls it before retrying an allocation."""
    with _POOL_LOCK:
        pool, width = _POOL
        if pool is None:
            return True
        return _release_pool(pool, width, timeout_s)


def _thread_stream(device):
    import torch

    ss = getattr(_TLS, "streams", None)
    if ss is None:
        ss = _TLS.streams = {}
    key = torch.device(device).index
    if key not in ss:
        ss[key] = torch.cuda.Stream(device)
    return ss[key]


class OneVsRestSVC:
    def __init__(self, C: float = 10.0, gamma: float = 0.00125, tol: float = 1e-5, eps: float = 1e-12,
                 sv_tol: float = 1e-8, max_iter: int = 100000, device: str = "auto", n_threads: int = 0,
                 gram: str = "auto", concurrent_solves: Optional[int] = None, solver: str = "auto",
                 wss: str = "first"):
        """``solver`` (GPU): "auto" = "decomp" unless ``wss="second"`` or a ``gram`` is forced, then
        "batched".  "batched" runs all pairwise class solves in ONE kernel launch over the shared Gram, a team
        of workgroups per XCD pulling classes from a queue; "streams" runs one persistent solve per
        class on ``concurrent_solves`` streams (default 8).  Results are identical either way.  "decomp":
        the working-set decomposition solver per class with no Gram, ``concurrent_solves`` classes at a time
        (default: all, or 2 past 192 MiB of pixel rows, where the solves are bound by passes over the rows).
        ``wss="second"``: the opt-in second-order working-set selection (as ``SVC(wss="second")``) in every class solve."""
        if solver not in ("auto", "batched", "streams", "decomp"):
            raise ValueError("solver must be auto, batched, streams or decomp")
        if solver == "decomp" and wss == "second":
            raise ValueError("the decomposition solver has its own (second-order) inner selection; wss applies to "
                             "the pairwise solvers")
        if wss not in ("first", "second"):
            raise ValueError("wss must be 'first' or 'second'")
        self.solver = solver
        self.concurrent_solves = concurrent_solves
        self._transport = None
        self.params = SVMParams(C=C, gamma=gamma, tau=tol, eps=eps, sv_tol=sv_tol, max_iter=max_iter,
                                n_threads=n_threads if n_threads > 0 else default_threads(),
                                wss=2 if wss == "second" else 1)
        self.device = device
        self.gram = gram

    def _dev(self) -> str:
        if self.device == "auto":
            import torch

            return "cuda" if torch.cuda.is_available() else "cpu"
        return self.device

    # ------------------------------------------------------------------ fit
    def fit(self, X: np.ndarray, labels: np.ndarray, classes: Optional[List[int]] = None,
            transport=None) -> "OneVsRestSVC":
        """With a ``transport`` (svm355.parallel.transport, e.g. one rank per GPU over RCCL) every rank
        passes the same rows, solves the classes k with k % world == rank on its own Gram, and the
        per-class alphas, b and iteration counts are all-reduced, so every rank ends with the whole
        model (identical to a single-rank fit)."""
        self._transport = transport
        cuda = self._dev() != "cpu"
        X = np.ascontiguousarray(X, dtype=np.uint8 if (cuda and X.dtype == np.uint8) else np.float64)
        labels = np.asarray(labels)
        self.classes_ = np.array(sorted(set(labels.tolist())) if classes is None else classes)
        self._n_pos = np.array([np.count_nonzero(labels == c) for c in self.classes_])  # per class
        t0 = time.perf_counter()
        if not cuda:
            self._fit_cpu(X, labels)
        else:
            self._fit_cuda(X, labels)
        self.fit_time_ = time.perf_counter() - t0
        return self

    def _ys(self, labels):
        return [np.where(labels == c, 1, -1).astype(np.int32) for c in self.classes_]

    def _mine(self, k: int) -> bool:
        t = self._transport
        return t is None or k % t.world == t.rank

    def _combine(self, alphas, bs, iters, stops):
        """All-reduce the per-class results of a distributed fit (zeros for other ranks' classes)."""
        t = self._transport
        if t is None:
            return alphas, bs, iters, stops
        import torch

        from .. import _native as N

        codes = {v: k for k, v in N.STOP_NAMES.items()}
        a = alphas if isinstance(alphas, torch.Tensor) else torch.from_numpy(alphas)
        meta = torch.tensor([[b, it, codes.get(st, 0)] for b, it, st in zip(bs, iters, stops)], dtype=torch.float64)
        a_c, m_c = a.to(t.device), meta.to(t.device)
        t.allreduce_(a_c, "sum")
        t.allreduce_(m_c, "sum")
        a = a_c.to(a.device)
        m = m_c.cpu().numpy()
        out_a = a if isinstance(alphas, torch.Tensor) else a.numpy()
        return (out_a, [float(x) for x in m[:, 0]], [int(x) for x in m[:, 1]],
                [N.STOP_NAMES.get(int(x), str(int(x))) for x in m[:, 2]])

    def _fit_cpu(self, X, labels):
        from ..ops import cpu as C

        self.scaler_ = MinMaxScaler().fit(X)
        check_finite_bounds(self.scaler_.min_, self.scaler_.max_)
        Xs = self.scaler_.transform(X)
        K = C.rbf_matrix(Xs, Xs, self.params.gamma, self.params.n_threads)
        ys = self._ys(labels)
        alphas = np.zeros((len(ys), X.shape[0]))
        bs, iters, stops = [0.0] * len(ys), [0] * len(ys), [""] * len(ys)
        for k, y in enumerate(ys):
            if not self._mine(k):
                continue
            a, r, _ = C.smo_train_gram(K, y, self.params)
            alphas[k], bs[k], iters[k], stops[k] = a, r.b, r.iterations, r.stop_reason
        alphas, bs, iters, stops = self._combine(alphas, bs, iters, stops)
        Y = np.stack(ys, 0)
        sup = np.flatnonzero((alphas > self.params.sv_tol).any(0)).astype(np.int64)
        self._finish(sup, (alphas * Y).T, bs, iters, stops)
        self.support_vectors_ = Xs[self.support_]
        self._dev_model = None

    def _fit_cuda(self, X, labels):
        import torch

        from ..ops import device as D

        device = torch.device(self._dev())
        if self.solver == "decomp" or (self.solver == "auto" and self.params.wss == 1 and self.gram == "auto"):
            return self._fit_cuda_decomp(X, labels, device)
        t0 = time.perf_counter()
        d = X.shape[1]
        Xu = K = None
        if X.dtype == np.uint8 and self.gram in ("auto", "int") and os.environ.get("SVM355_U8_TRAIN", "1") != "0":
            # byte path (as SVC._fit_cuda_u8): min/max, quantisation and Gram from the device bytes
            Xu = D.upload_u8(X, device)
            mn, mx = D.minmax_u8(Xu)
            mm = torch.cat([mn, mx]).cpu().numpy()
            mn_h, mx_h = mm[:d].copy(), mm[d:].copy()
            t1 = time.perf_counter()
            with trace_range("svm355.ovr.gram"):
                K = D.rbf_gram_u8(Xu, self.params.gamma, mn_h, mx_h, out=D.gram_buffer(X.shape[0], device))
            path = "int8-exact"
        if K is None:
            Xu = None
            t0 = time.perf_counter()
            Xd = D.upload_rows(X, device)
            mn, mx, sqn = D.minmax_scale_(Xd, d)
            check_finite_bounds(mn.cpu().numpy(), mx.cpu().numpy())
            t1 = time.perf_counter()
            K, path = D.rbf_gram_sym(Xd, sqn, self.params.gamma, mn=mn, mx=mx, gram=self.gram,
                                     out=D.gram_buffer(X.shape[0], device))
        torch.cuda.synchronize(device)
        t2 = time.perf_counter()
        n = X.shape[0]
        alphas = torch.zeros((len(self.classes_), n), dtype=torch.float64, device=device)
        ys = self._ys(labels)
        ys_d = [torch.from_numpy(y).to(device) for y in ys]
        torch.cuda.synchronize(device)

        def solve(k):
            # Each class solve on its own stream (and, per host thread, its own device context):
            # the SMO is latency-bound on <= 64 workgroups, so several classes share the 256 CUs.
            s = torch.cuda.Stream(device)
            with torch.cuda.stream(s):
                r, _ = D.smo(K, ys_d[k], alphas[k], self.params, n=n)
            s.synchronize()
            return r

        mine = [k for k in range(len(ys)) if self._mine(k)]
        results = {}
        self.batched_ = False
        with trace_range(f"svm355.ovr.solve classes={len(mine)}"):
            if self.solver in ("auto", "batched") and mine:
                # One launch: an XCD-local team per XCD, classes pulled from a queue (smo_multi_kernel).
                Yb = torch.stack([ys_d[k] for k in mine]).contiguous()
                Ab = torch.zeros((len(mine), n), dtype=torch.float64, device=device)
                rs, self.batched_ = D.smo_multi(K, Yb, Ab, self.params, n=n)
                alphas[mine] = Ab
                results = dict(zip(mine, rs))
            workers = max(1, min(self.concurrent_solves or 8, len(mine)))
            if results:
                pass
            elif workers > 1:
                from concurrent.futures import ThreadPoolExecutor

                with ThreadPoolExecutor(max_workers=workers) as ex:  # the native calls release the GIL
                    results = dict(zip(mine, ex.map(solve, mine)))
            else:
                results = {k: solve(k) for k in mine}
            bs = [results[k].b if k in results else 0.0 for k in range(len(ys))]
            iters = [results[k].iterations if k in results else 0 for k in range(len(ys))]
            stops = [results[k].stop_reason if k in results else "" for k in range(len(ys))]
            torch.cuda.synchronize(device)
        alphas, bs, iters, stops = self._combine(alphas, bs, iters, stops)
        t3 = time.perf_counter()
        del K
        a = alphas.cpu().numpy()  # (classes, n)
        Y = np.stack(ys, 0)
        sup = np.flatnonzero((a > self.params.sv_tol).any(0)).astype(np.int64)
        self._finish(sup, (a * Y).T, bs, iters, stops)
        idx = torch.from_numpy(self.support_).to(device)
        Xs, ns = D.sv_rows_u8(Xu, idx, mn, mx) if Xu is not None else (D.gather_rows(Xd, idx), sqn[idx].contiguous())
        self._dev_model = {"Xs": Xs, "ns": ns,
                           "coef": torch.from_numpy(np.ascontiguousarray(self.dual_coef_)).to(device),
                           "b": torch.tensor(self.intercepts_b_, dtype=torch.float64, device=device),
                           "mn": mn, "mx": mx, "d": d, "device": device}
        self.scaler_ = MinMaxScaler(mn.cpu().numpy(), mx.cpu().numpy())
        self.timings_ = {"upload_preprocess_ms": (t1 - t0) * 1e3, "gram_ms": (t2 - t1) * 1e3,
                         "smo_ms_all_classes": (t3 - t2) * 1e3, "gram_path": path,
                         "smo_solver": "batched" if self.batched_ else "streams"}

    def _fit_cuda_decomp(self, X, labels, device):
        """Every class by the decomposition solver on the shared device rows (no Gram)."""
        import torch

        from .. import _native as N
        from ..ops import device as D

        t0 = time.perf_counter()
        d = X.shape[1]
        Xu = Xd = sqn = None
        if X.dtype == np.uint8:
            Xu = D.upload_u8(X, device)
            mn, mx = D.minmax_u8(Xu)
            rows = Xu
        else:
            Xd = D.upload_rows(X, device)
            mn, mx, sqn = D.minmax_scale_(Xd, d)
            check_finite_bounds(mn.cpu().numpy(), mx.cpu().numpy())
            rows = Xd
        mm = torch.cat([mn, mx]).cpu().numpy()
        mn_h, mx_h = mm[:d].copy(), mm[d:].copy()
        t1 = time.perf_counter()
        n = X.shape[0]
        ys = self._ys(labels)
        ys_d = [torch.from_numpy(y).to(device) for y in ys]
        alphas = torch.zeros((len(self.classes_), n), dtype=torch.float64, device=device)
        torch.cuda.synchronize(device)
        mine = [k for k in range(len(ys)) if self._mine(k)]

        # all classes side by side while the rows sit in the last-level cache (the solves are bound by their
        # one-CU inner chains); past 192 MiB of pixel rows (where the column cache turns on) they are bound
        # by HBM passes over the rows and two at a time is fastest (1M: 5.7 s against 7.6 s one at a time
        # and 9-14 s all ten, profiles/r5_ovr_large_n.txt)
        big = X.shape[0] * X.shape[1] > (192 << 20)
        workers = self.concurrent_solves or (2 if big else len(mine))
        width = min(workers, max(1, len(mine)))
        # Large n: every solving thread's context keeps one column-cache slab for all its classes and for the
        # next fit -- freeing and re-allocating a tens-of-GB slab made the later solves' caches 2-7x slower
        # per outer iteration (per class, and again per fit: profiles/r5_ovr_large_n.txt) -- the slabs of a
        # pool together capped at half the HBM; release_solver_caches() hands them back.
        frac = min(0.25, 0.5 / width)

        def solve(k):
            s = _thread_stream(device)
            ctx = D.DeviceContext.get(device)
            N.check(ctx.lib.svmd_set_ccache_frac(ctx.handle, frac), "svmd_set_ccache_frac")
            with torch.cuda.stream(s):
                out = D.train_decomp(rows, ys_d[k], alphas[k], self.params, mn_h, mx_h)
            s.synchronize()
            if out is None:
                raise N.NativeError(f"class {self.classes_[k]}: the decomposition solver declined these rows "
                                    "(no exact-integer plan for uint8 rows, or beyond its shapes); use "
                                    "solver='batched'")
            return out

        with trace_range(f"svm355.ovr.decomp classes={len(mine)}"):
            outs = dict(zip(mine, _pool(width).map(solve, mine))) if mine else {}
            torch.cuda.synchronize(device)
        bs = [outs[k][0].b if k in outs else 0.0 for k in range(len(ys))]
        iters = [outs[k][0].iterations if k in outs else 0 for k in range(len(ys))]
        stops = [outs[k][0].stop_reason if k in outs else "" for k in range(len(ys))]
        alphas, bs, iters, stops = self._combine(alphas, bs, iters, stops)
        t2 = time.perf_counter()
        a = alphas.cpu().numpy()
        Y = np.stack(ys, 0)
        sup = np.flatnonzero((a > self.params.sv_tol).any(0)).astype(np.int64)
        self._finish(sup, (a * Y).T, bs, iters, stops)
        idx = torch.from_numpy(self.support_).to(device)
        Xs, ns = D.sv_rows_u8(Xu, idx, mn, mx) if Xu is not None else (D.gather_rows(Xd, idx), sqn[idx].contiguous())
        self._dev_model = {"Xs": Xs, "ns": ns,
                           "coef": torch.from_numpy(np.ascontiguousarray(self.dual_coef_)).to(device),
                           "b": torch.tensor(self.intercepts_b_, dtype=torch.float64, device=device),
                           "mn": mn, "mx": mx, "d": d, "device": device}
        self.scaler_ = MinMaxScaler(mn_h, mx_h)
        self.batched_ = False
        self.class_timings_ = {int(self.classes_[k]): outs[k][1] for k in outs}
        self.timings_ = {"upload_preprocess_ms": (t1 - t0) * 1e3, "gram_ms": 0.0,
                         "smo_ms_all_classes": (t2 - t1) * 1e3, "gram_path": "none (decomposition)",
                         "smo_solver": "decomp"}

    def _finish(self, sup, coef_full, bs, iters, stops):
        # a class absent from the labels (or covering them all) has no violating pair: its solve stops with
        # no candidate and alpha = 0; make it the constant predictor -1 (or +1) instead of decision 0 - b = 0,
        # which would outrank every real class whose decision values are negative
        bs = list(bs)
        n_rows = len(coef_full)
        for c, pos in enumerate(self._n_pos):
            if pos == 0 or pos == n_rows:
                bs[c] = 1.0 if pos == 0 else -1.0
        self.support_ = sup
        self.dual_coef_ = np.ascontiguousarray(coef_full[sup])  # (n_sv_union, classes)
        self.intercepts_b_ = np.asarray(bs, dtype=np.float64)  # per-class b (decision = K coef - b)
        self.n_iter_ = np.asarray(iters)
        self.stop_reasons_ = list(stops)

    # ------------------------------------------------------------------ persistence
    def _host_sv_rows(self) -> np.ndarray:
        """The union support vectors' scaled rows on the host (from the device model after a GPU fit)."""
        if self._dev_model is not None:
            dm = self._dev_model
            return np.ascontiguousarray(dm["Xs"][:, : dm["d"]].cpu().numpy())
        return np.ascontiguousarray(self.support_vectors_)

    def save(self, directory) -> None:
        """One directory per class with the reference's model files (``final_sv_ids.txt``,
        ``final_sv_labels.txt``, ``final_sv_alphas.txt``, ``final_b.txt``: the class's nonzero dual
        coefficients over the union of support vectors, ids = training rows), plus the union's scaled rows
        (``sv_rows.npy``), the scaler (``scaler.npz``) and ``ovr.json`` -- pickle-free throughout."""
        import json
        from pathlib import Path

        from .model_io import save_model

        d = Path(directory)
        d.mkdir(parents=True, exist_ok=True)
        np.save(d / "sv_rows.npy", self._host_sv_rows(), allow_pickle=False)
        np.save(d / "support.npy", np.ascontiguousarray(self.support_, dtype=np.int64), allow_pickle=False)
        if self.scaler_ is not None:
            np.savez(d / "scaler.npz", min=self.scaler_.min_, max=self.scaler_.max_)
        for c, label in enumerate(self.classes_):
            coef = self.dual_coef_[:, c]
            nz = np.flatnonzero(coef != 0.0)
            save_model(d / f"class_{label}", ids=self.support_[nz], labels=np.where(coef[nz] > 0, 1, -1),
                       alphas=np.abs(coef[nz]), b=float(self.intercepts_b_[c]), params=self.params,
                       meta={"class": int(label), "n_iter": int(self.n_iter_[c]), "stop_reason": self.stop_reasons_[c]})
        (d / "ovr.json").write_text(json.dumps({"format": "svm355-ovr-v1", "classes": [int(x) for x in self.classes_],
                                                "n_sv_union": int(len(self.support_)), "params": self.params.as_dict()},
                                               indent=2))

    @classmethod
    def load(cls, directory, device: str = "cpu") -> "OneVsRestSVC":
        """The model ``save`` wrote; ``device`` "cuda[:k]" keeps the SV rows on that GPU for prediction."""
        import json
        from pathlib import Path

        from ..utils.config import SVMParams
        from .model_io import load_model

        d = Path(directory)
        info = json.loads((d / "ovr.json").read_text())
        p = SVMParams(**info["params"])
        m = cls(C=p.C, gamma=p.gamma, tol=p.tau, eps=p.eps, sv_tol=p.sv_tol, max_iter=p.max_iter, device=device,
                wss="second" if p.wss == 2 else "first")
        m.classes_ = np.array(info["classes"])
        m.support_ = np.load(d / "support.npy", allow_pickle=False)
        m.support_vectors_ = np.load(d / "sv_rows.npy", allow_pickle=False)
        m.scaler_ = None
        if (d / "scaler.npz").exists():
            z = np.load(d / "scaler.npz", allow_pickle=False)
            m.scaler_ = MinMaxScaler(z["min"], z["max"])
        coef = np.zeros((len(m.support_), len(m.classes_)))
        bs, iters, stops = [], [], []
        for c, label in enumerate(m.classes_):
            mc = load_model(d / f"class_{label}")
            pos = np.searchsorted(m.support_, mc["ids"])
            if len(pos) and (pos.max() >= len(m.support_) or np.any(m.support_[pos] != mc["ids"])):
                raise ValueError(f"class {label}: support vector ids outside the saved union")
            coef[pos, c] = mc["alphas"] * mc["labels"]
            bs.append(mc["b"])
            meta = json.loads((d / f"class_{label}" / "model.json").read_text()).get("meta", {})
            iters.append(int(meta.get("n_iter", 0)))
            stops.append(meta.get("stop_reason", ""))
        m.dual_coef_ = coef
        m.intercepts_b_ = np.asarray(bs, dtype=np.float64)
        m.n_iter_ = np.asarray(iters)
        m.stop_reasons_ = stops
        m._dev_model = None
        if m._dev() != "cpu":
            if m.scaler_ is None:
                raise ValueError("a device model needs the saved scaler (scaler.npz)")
            import torch

            from ..ops import device as D

            dev = torch.device(m._dev())
            k, dd = m.support_vectors_.shape
            Xs = D.upload_rows(m.support_vectors_, dev)
            mm = np.concatenate([m.scaler_.min_, m.scaler_.max_]).astype(np.float64)
            mmd = torch.from_numpy(mm).to(dev)
            m._dev_model = {"Xs": Xs, "ns": D.row_norms(Xs, dd),
                            "coef": torch.from_numpy(np.ascontiguousarray(coef)).to(dev),
                            "b": torch.tensor(m.intercepts_b_, dtype=torch.float64, device=dev),
                            "mn": mmd[:dd], "mx": mmd[dd:], "d": dd, "device": dev}
        return m

    # ------------------------------------------------------------------ inference
    def decision_function(self, X: np.ndarray) -> np.ndarray:
        """(m, classes) decision values sum_k coef_kc K(x, sv_k) - b_c."""
        d = (int(self._dev_model["d"]) if self._dev_model is not None else
             int(np.size(self.scaler_.min_)) if self.scaler_ is not None else int(np.shape(self.support_vectors_)[1]))
        if np.ndim(X) != 2 or np.shape(X)[1] != d:
            raise ValueError(f"X must be (m, {d}) like the training rows, got shape {np.shape(X)}")
        X = np.ascontiguousarray(X, dtype=np.uint8 if (self._dev_model is not None and X.dtype == np.uint8)
                                 else np.float64)
        if self._dev_model is not None:
            import torch

            from ..ops import device as D

            dm = self._dev_model
            Xq = D.upload_rows(X, dm["device"])
            _, _, nq = D.minmax_scale_(Xq, dm["d"], dm["mn"], dm["mx"])
            Kq = D.rbf_gram(Xq, nq, dm["Xs"], dm["ns"], self.params.gamma)[:, : dm["Xs"].shape[0]]
            return (torch.matmul(Kq, dm["coef"]) - dm["b"]).cpu().numpy()
        from ..ops import cpu as C

        Xq = self.scaler_.transform(X)
        Kq = C.rbf_matrix(Xq, self.support_vectors_, self.params.gamma, self.params.n_threads)
        return Kq @ self.dual_coef_ - self.intercepts_b_

    def predict(self, X: np.ndarray) -> np.ndarray:
        return self.classes_[np.argmax(self.decision_function(X), axis=1)]

    def score(self, X: np.ndarray, labels: np.ndarray) -> float:
        return float(np.mean(self.predict(X) == np.asarray(labels)))
