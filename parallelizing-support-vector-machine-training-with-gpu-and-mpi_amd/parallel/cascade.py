"""Cascade SVM over data-parallel ranks (one rank per MI355X GPU, or CPU/thread ranks for tests).

Two topologies, both with the reference's round structure, warm starts, ID de-duplication and
ID-set convergence test:

``topology="tree"`` — classical Cascade (mpi_svm_main3.cpp:565-828), P a power of two.
    Each round: rank 0's SV set from the last round (with alphas) is broadcast; at step = 1 every
    rank trains on (broadcast SVs, warm alphas) U (its partition rows not in that set, alpha = 0);
    then for step = 2, 4, ..., P the rank ``r % step == 0`` trains on (SVs received from
    ``r + step/2``... i.e. its partner, warm) U (its own current SVs not among them, alpha = 0) after
    senders ``r % 2step == step`` ship their SVs to ``r - step``.  Rank 0's final-layer SVs become
    the global set; the round converges when their ID set equals the previous round's.

``topology="star"`` — modified two-layer Cascade (mpi_svm_main2.cpp:439-769), any P.
    Each round: the global SV set is broadcast; every rank trains on (global SVs, warm) U (its
    partition rows not in it, alpha = 0); local SVs are gathered to rank 0, which merges its own SVs
    (alphas kept) with the workers' unseen SVs in rank order (alphas reset to 0, :600-601), retrains,
    and takes the result as the next global set; convergence = same ID set.

Everything stays on the rank's device: partitions are scaled in place with globally all-reduced
min/max (bitwise identical to the reference's rank-0 min/max + broadcast, M3 :529-539), SV sets
travel as one packed float64 buffer per exchange (transport.py), and every local solve is the
device SMO with a warm-start f computed from the resident RBF Gram.  Rank-0 stdout lines follow
the reference's; timing starts after data distribution as in M3 :526.
"""
from __future__ import annotations

import json
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable, List, Optional

import numpy as np
import torch

from ..utils.config import SVMParams
from ..utils.trace import trace_range
from .transport import Transport


# ---------------------------------------------------------------------------------------- backends
class _CpuBackend:
    """Native C++ oracle solver; rows are CPU tensors of width d."""

    name = "cpu"

    def __init__(self, params: SVMParams, d: int):
        self.params = params
        self.d = d
        self.width = d

    def to_rows(self, X: np.ndarray, device) -> torch.Tensor:
        # Always a private copy: rows are scaled in place and must not alias the caller's array.
        return torch.from_numpy(np.array(X, dtype=np.float64, order="C", copy=True))

    def local_minmax(self, X: torch.Tensor):
        from ..utils.data import MinMaxScaler

        s = MinMaxScaler().fit(X.numpy())
        return torch.from_numpy(s.min_), torch.from_numpy(s.max_)

    def scale_(self, X: torch.Tensor, mn: torch.Tensor, mx: torch.Tensor) -> None:
        from ..utils.data import MinMaxScaler

        if X.shape[0]:
            X.copy_(torch.from_numpy(MinMaxScaler(mn.numpy(), mx.numpy()).transform(X.numpy())))

    def solve(self, X: torch.Tensor, y: np.ndarray, alpha: np.ndarray):
        from ..ops import cpu as C

        a, res, _ = C.smo_train(X.numpy(), y, self.params, alpha=alpha, warm=True)
        return a, res

    def select(self, X: torch.Tensor, idx: np.ndarray) -> torch.Tensor:
        return X[torch.from_numpy(np.asarray(idx, dtype=np.int64))]

    def decision(self, sv_X: torch.Tensor, coef: np.ndarray, y_sv: np.ndarray, alpha_sv: np.ndarray,
                 Xq: torch.Tensor, b: float) -> np.ndarray:
        from ..ops import cpu as C

        return C.decision(sv_X.numpy(), y_sv, alpha_sv, Xq.numpy(), self.params.gamma, b, self.params.n_threads)

    def sync(self):
        pass


class _HipBackend:
    """gfx950 device solver; rows are (k, ld) float64 device tensors, ld = round_up(d, 16)."""

    name = "hip"

    def __init__(self, params: SVMParams, d: int, device: torch.device):
        from ..ops import device as D

        self.D = D
        self.params = params
        self.d = d
        self.width = D.padded_dim(d)
        self.device = device
        self.stats = None  # host (min, max) the rows were scaled with -> exact-integer Gram path

    def to_rows(self, X: np.ndarray, device) -> torch.Tensor:
        return self.D.upload_rows(X, self.device, self.width)

    def local_minmax(self, X: torch.Tensor):
        # Local column min/max; the caller all-reduces them and then scales (use_given path).
        if X.shape[0] == 0:
            return (torch.full((self.d,), float("inf"), dtype=torch.float64, device=self.device),
                    torch.full((self.d,), float("-inf"), dtype=torch.float64, device=self.device))
        return self.D.minmax(X, self.d)

    def scale_(self, X: torch.Tensor, mn: torch.Tensor, mx: torch.Tensor) -> None:
        if self.stats is None:
            self.stats = (mn.detach().cpu().numpy().copy(), mx.detach().cpu().numpy().copy())
        if X.shape[0]:
            self.D.minmax_scale_(X, self.d, mn, mx)

    def solve(self, X: torch.Tensor, y: np.ndarray, alpha: np.ndarray):
        D = self.D
        m = X.shape[0]
        sqn = D.row_norms(X, self.d)
        yd = torch.from_numpy(np.ascontiguousarray(y, dtype=np.int32)).to(self.device)
        ad = torch.from_numpy(np.ascontiguousarray(alpha, dtype=np.float64)).to(self.device)
        mn, mx = self.stats if self.stats is not None else (None, None)
        res, _ = D.train(X, sqn, yd, ad, self.params, warm=True, K=D.gram_buffer(m, self.device), mn=mn, mx=mx)
        return ad.cpu().numpy(), res

    def select(self, X: torch.Tensor, idx: np.ndarray) -> torch.Tensor:
        return self.D.gather_rows(X, torch.from_numpy(np.asarray(idx, dtype=np.int64)))

    def decision(self, sv_X, coef, y_sv, alpha_sv, Xq, b):
        return self.decision_device(sv_X, coef, Xq, b).cpu().numpy()

    def decision_device(self, sv_X, coef, Xq, b) -> torch.Tensor:
        D = self.D
        ns = D.row_norms(sv_X, self.d)
        nq = D.row_norms(Xq, self.d)
        c = torch.from_numpy(np.ascontiguousarray(coef)).to(self.device)
        return D.decision(sv_X, ns, c, Xq, nq, self.params.gamma, b)

    def count_correct(self, dec: torch.Tensor, y: np.ndarray) -> int:
        return self.D.count_correct(dec, y, zero_is_positive=True)  # s >= 0 -> +1 (M3 :800)

    def sync(self):
        torch.cuda.synchronize(self.device)


# ---------------------------------------------------------------------------------------- SV sets
@dataclass
class SVSet:
    X: torch.Tensor  # (k, w) scaled rows on the rank's device
    y: np.ndarray  # (k,) int32 +-1
    alpha: np.ndarray  # (k,) float64
    ids: np.ndarray  # (k,) int64 global sample ids

    def __len__(self) -> int:
        return int(self.ids.shape[0])

    @staticmethod
    def empty(width: int, device) -> "SVSet":
        return SVSet(torch.empty((0, width), dtype=torch.float64, device=device), np.empty(0, np.int32),
                     np.empty(0, np.float64), np.empty(0, np.int64))

    def pack(self) -> torch.Tensor:
        dev = self.X.device
        cols = torch.from_numpy(np.stack([self.y.astype(np.float64), self.alpha, self.ids.astype(np.float64)], 1)
                                if len(self) else np.empty((0, 3))).to(dev)
        return torch.cat([self.X, cols], dim=1).contiguous()

    @staticmethod
    def unpack(t: torch.Tensor, width: int) -> "SVSet":
        tail = t[:, width:].cpu().numpy()
        return SVSet(t[:, :width].contiguous(), tail[:, 0].astype(np.int32), tail[:, 1].copy(),
                     tail[:, 2].astype(np.int64))

    def id_set(self) -> set:
        return set(self.ids.tolist())


def _concat(backend, a: SVSet, b: SVSet) -> SVSet:
    return SVSet(torch.cat([a.X, b.X], 0) if len(b) else a.X, np.concatenate([a.y, b.y]),
                 np.concatenate([a.alpha, b.alpha]), np.concatenate([a.ids, b.ids]))


def _subset(backend, s: SVSet, idx: np.ndarray, zero_alpha: bool = False) -> SVSet:
    idx = np.asarray(idx, dtype=np.int64)
    return SVSet(backend.select(s.X, idx), s.y[idx], np.zeros(len(idx)) if zero_alpha else s.alpha[idx],
                 s.ids[idx])


def merge_unseen(backend, warm: SVSet, extra: SVSet) -> SVSet:
    """warm (alphas kept) U rows of extra whose id is not in warm (alpha = 0), extra order kept.
    Reference: the seen_ids loops of mpi_svm_main3.cpp:629-655 / mpi_svm_main2.cpp:474-502."""
    if len(warm) == 0:
        return _subset(backend, extra, np.arange(len(extra)), zero_alpha=True)
    keep = np.flatnonzero(~np.isin(extra.ids, warm.ids))
    return _concat(backend, warm, _subset(backend, extra, keep, zero_alpha=True))


# ---------------------------------------------------------------------------------------- results
@dataclass
class CascadeResult:
    sv: SVSet
    b: float
    rounds: int
    converged: bool
    sv_history: List[int] = field(default_factory=list)
    merged_history: List[int] = field(default_factory=list)
    round_ms: List[float] = field(default_factory=list)
    train_ms: float = 0.0
    solves: List[dict] = field(default_factory=list)
    mn: Optional[torch.Tensor] = None
    mx: Optional[torch.Tensor] = None


class CascadeSVM:
    """Rank-local (SPMD) Cascade SVM driver; every rank of ``transport`` calls :meth:`fit`."""

    def __init__(self, transport: Transport, params: Optional[SVMParams] = None, topology: str = "star",
                 max_rounds: int = 50, backend: str = "auto", verbose: int = 1,
                 log: Optional[Callable[[str], None]] = None, checkpoint_dir: Optional[str] = None,
                 resume: bool = False, device=None):
        """``device`` is where rows live and solves run (default: the transport's device).  A
        compute device different from the transport's (e.g. GPU compute with a gloo CPU group)
        stages every exchanged buffer through the transport device."""
        if topology not in ("star", "tree"):
            raise ValueError("topology must be 'star' (modified two-layer) or 'tree' (classical)")
        self.t = transport
        self.device = torch.device(device) if device is not None else transport.device
        self.params = params or SVMParams()
        self.topology = topology
        self.max_rounds = max_rounds
        self.backend_name = backend
        self.verbose = verbose
        self._log = log or (lambda s: print(s, flush=True))
        self.checkpoint_dir = Path(checkpoint_dir) if checkpoint_dir else None
        self.resume = resume
        self.result: Optional[CascadeResult] = None
        if topology == "tree" and (self.t.world & (self.t.world - 1)):
            # mpi_svm_main3.cpp:420-428 aborts on a non-power-of-2 communicator.
            raise ValueError(f"classical (tree) cascade needs a power-of-2 number of ranks, got {self.t.world}")

    # ------------------------------------------------------------------ helpers
    def log(self, msg: str, level: int = 1) -> None:
        if self.t.rank == 0 and self.verbose >= level:
            self._log(msg)

    # ---- communication helpers (stage through the transport device when it differs)
    def _c(self, x: torch.Tensor) -> torch.Tensor:
        return x if x.device == self.t.device else x.to(self.t.device)

    def _d(self, x: torch.Tensor) -> torch.Tensor:
        return x if x.device == self.device else x.to(self.device)

    def _bcast_set(self, S: Optional[SVSet], width: int) -> SVSet:
        with trace_range("cascade:bcast_svs"):
            payload = self._c(S.pack()) if self.t.rank == 0 else None
            return SVSet.unpack(self._d(self.t.broadcast_rows(payload, width + 3)), width)

    def _allreduce(self, x: torch.Tensor, op: str) -> torch.Tensor:
        y = self._c(x.clone())
        self.t.allreduce_(y, op)
        return self._d(y)

    def _make_backend(self, d: int):
        dev = self.device
        name = self.backend_name
        if name == "auto":
            name = "hip" if dev.type == "cuda" else "cpu"
        if name == "hip":
            return _HipBackend(self.params, d, dev)
        return _CpuBackend(self.params, d)

    def _solve(self, be, S: SVSet, tag: str, rnd: int, res_log: list) -> SVSet:
        """Warm-start SMO on S (SMO_train(..., init=false)); returns its SVs (alpha > sv_tol)."""
        if len(S) == 0:
            return S, 0.0
        t0 = time.perf_counter()
        with trace_range(f"cascade:solve:{tag}"):
            alpha, res = be.solve(S.X, S.y, S.alpha)
        dt = (time.perf_counter() - t0) * 1e3
        res_log.append({"round": rnd, "rank": self.t.rank, "layer": tag, "n": len(S), "iterations": res.iterations,
                        "b": res.b, "stop": res.stop_reason, "ms": dt})
        if self.verbose >= 2:
            print(f"[rank {self.t.rank}] round {rnd} {tag}: n={len(S)} iterations={res.iterations} b={res.b:.15f} "
                  f"stop={res.stop_reason} {dt:.1f} ms", flush=True)
        keep = np.flatnonzero(alpha > self.params.sv_tol)
        out = SVSet(be.select(S.X, keep), S.y[keep], alpha[keep], S.ids[keep])
        return out, res.b

    def _checkpoint(self, rnd: int, G: SVSet, b: float, global_ids) -> None:
        if self.checkpoint_dir is None or self.t.rank != 0:
            return
        self.checkpoint_dir.mkdir(parents=True, exist_ok=True)
        tmp = self.checkpoint_dir / "cascade_state.tmp.npz"
        np.savez(tmp, round=rnd, b=b, sv=G.pack().cpu().numpy(), width=G.X.shape[1],
                 global_ids=np.asarray(sorted(global_ids), dtype=np.int64), topology=self.topology)
        tmp.replace(self.checkpoint_dir / "cascade_state.npz")

    def _load_checkpoint(self, be):
        path = self.checkpoint_dir / "cascade_state.npz" if self.checkpoint_dir else None
        has = int(self.t.rank == 0 and path is not None and self.resume and path.exists())
        has = self.t.broadcast_int(has)
        if not has:
            return None
        if self.t.rank == 0:
            z = np.load(path, allow_pickle=False)
            if int(z["width"]) != be.width or str(z["topology"]) != self.topology:
                raise ValueError("checkpoint does not match this cascade configuration")
            payload = torch.from_numpy(z["sv"]).to(self.t.device)
            rnd, b, gids = int(z["round"]), float(z["b"]), set(z["global_ids"].tolist())
        else:
            payload, rnd, b, gids = None, 0, 0.0, set()
        rnd = self.t.broadcast_int(rnd)
        G = SVSet.unpack(self._d(self.t.broadcast_rows(payload, be.width + 3)), be.width)
        return rnd, b, G, gids

    # ------------------------------------------------------------------ fit
    def fit(self, X_part: np.ndarray, y_part: np.ndarray, ids_part: np.ndarray, n_total: Optional[int] = None
            ) -> CascadeResult:
        """Train on this rank's partition (raw, unscaled rows) with global sample ids."""
        t = self.t
        # uint8 pixel rows stay compact up to the device (widened to FP64 there)
        X_part = np.ascontiguousarray(X_part, dtype=np.uint8 if X_part.dtype == np.uint8 else np.float64)
        d = t.broadcast_int(X_part.shape[1] if t.rank == 0 else 0)
        if X_part.shape[1] != d:
            raise ValueError(f"rank {t.rank}: partition has {X_part.shape[1]} features, rank 0 has {d}")
        n_total = t.broadcast_int(n_total if n_total is not None else 0)
        be = self._make_backend(d)
        name = "modified CascadeSVM" if self.topology == "star" else "CascadeSVM"
        self.log(f"[rank 0] Running {name} with {t.world} processes")
        if n_total:
            self.log(f"[rank 0] total samples = {n_total}, features = {d}")
        part = SVSet(be.to_rows(X_part, self.device), np.ascontiguousarray(y_part, np.int32),
                     np.zeros(X_part.shape[0]), np.ascontiguousarray(ids_part, np.int64))
        be.sync()
        t.barrier()

        t0 = time.perf_counter()  # M3 :526 — after data distribution, before scaling
        mn, mx = be.local_minmax(part.X)
        mn = self._allreduce(mn, "min")
        mx = self._allreduce(mx, "max")
        be.scale_(part.X, mn, mx)

        solves: list = []
        res = CascadeResult(SVSet.empty(be.width, self.device), 0.0, 0, False, mn=mn, mx=mx)
        G = SVSet.empty(be.width, self.device)  # global SV set (meaningful on rank 0; broadcast each round)
        global_ids: set = set()
        b = 0.0
        start_round = 0
        ck = self._load_checkpoint(be)
        if ck is not None:
            start_round, b, G, global_ids = ck
            self.log(f"[rank 0] resumed from checkpoint at round {start_round}, SV count = {len(G)}")
        tr_prev = time.perf_counter()
        rnd = start_round
        converged = False
        while rnd < self.max_rounds and not converged:
            shown = rnd if self.topology == "star" else rnd + 1
            round_range = trace_range(f"cascade:round{shown}")
            round_range.__enter__()
            self.log(f"=== Round {shown} ===")
            # Broadcast the global SV set (count + one packed buffer) from rank 0.
            G = self._bcast_set(G, be.width)
            if self.topology == "star":
                S = merge_unseen(be, G, part)
                local, _ = self._solve(be, S, "local", shown, solves)
                with trace_range("cascade:gather_svs"):
                    gathered = t.gather_rows(self._c(local.pack()), dst=0)
                same = 0
                if t.rank == 0:
                    merged = local
                    seen = set(local.ids.tolist())
                    for src in range(1, t.world):  # source order 1..P-1 (M2 :578)
                        w = SVSet.unpack(self._d(gathered[src]), be.width)
                        keep = [i for i, g in enumerate(w.ids.tolist()) if g not in seen]
                        seen.update(w.ids[keep].tolist())
                        merged = _concat(be, merged, _subset(be, w, np.asarray(keep, np.int64), zero_alpha=True))
                    res.merged_history.append(len(merged))
                    self.log(f"[rank 0] merged unique SV count from workers = {len(merged)}")
                    newG, b = self._solve(be, merged, "merge", shown, solves)
                    new_ids = newG.id_set()
                    same = int(len(newG) == len(global_ids) and new_ids == global_ids)
                    G, global_ids = newG, new_ids
                    be.sync()
                    tr = time.perf_counter()
                    res.round_ms.append((tr - tr_prev) * 1e3)
                    self.log(f"[rank 0] Round{shown} takes {int((tr - tr_prev) * 1e3)} ms")
                    tr_prev = tr
            else:
                cur = part
                recv = G
                step = 1
                while step <= t.world:
                    if t.rank % step == 0:
                        S = merge_unseen(be, recv, cur)
                        cur, b_local = self._solve(be, S, f"layer{step}", shown, solves)
                        if t.rank == 0:
                            b = b_local
                    if step < t.world:
                        if t.rank % (2 * step) == step:
                            with trace_range(f"cascade:send_svs:step{step}"):
                                t.send_rows(self._c(cur.pack()), t.rank - step)
                        elif t.rank % (2 * step) == 0:
                            with trace_range(f"cascade:recv_svs:step{step}"):
                                recv = SVSet.unpack(self._d(t.recv_rows(t.rank + step, be.width + 3)), be.width)
                    step *= 2
                same = 0
                if t.rank == 0:
                    new_ids = cur.id_set()
                    same = int(len(cur) == len(global_ids) and new_ids == global_ids)
                    G, global_ids = cur, new_ids
                    be.sync()
                    tr = time.perf_counter()
                    res.round_ms.append((tr - tr_prev) * 1e3)
                    tr_prev = tr
            if t.rank == 0:
                res.sv_history.append(len(G))
                if same:
                    self.log(f"[rank 0] Converged at round {shown}, SV count = {len(G)}")
                else:
                    self.log(f"[rank 0] Not converged yet. New SV count = {len(G)}")
                self._checkpoint(rnd + 1, G, b, global_ids)
            converged = bool(t.broadcast_int(same))
            round_range.__exit__(None, None, None)
            rnd += 1

        # Share the final model with every rank (the reference keeps it on rank 0 only).
        b_t = torch.tensor([b], dtype=torch.float64, device=t.device)
        t.broadcast_(b_t, 0)
        G = self._bcast_set(G, be.width)
        be.sync()
        t1 = time.perf_counter()
        res.sv, res.b, res.rounds, res.converged = G, float(b_t.item()), rnd, converged
        res.train_ms = (t1 - t0) * 1e3
        res.solves = solves
        self.log(f"[rank 0] Final b = {res.b:.15f}")
        self.result = res
        self._be = be
        return res

    # ------------------------------------------------------------------ inference
    def decision_function(self, X: np.ndarray) -> np.ndarray:
        r, be = self.result, self._be
        X = np.ascontiguousarray(X, dtype=np.uint8 if X.dtype == np.uint8 else np.float64)
        Xq = be.to_rows(X, self.device)
        be.scale_(Xq, r.mn, r.mx)
        if len(r.sv) == 0:
            return np.full(X.shape[0], -r.b)
        return be.decision(r.sv.X, r.sv.alpha * r.sv.y, r.sv.y, r.sv.alpha, Xq, r.b)

    def predict(self, X: np.ndarray, zero_is_positive: bool = True) -> np.ndarray:
        """Cascade programs map s >= 0 to +1 (M3 :800, M2 :729)."""
        dec = self.decision_function(X)
        return np.where(dec >= 0 if zero_is_positive else dec > 0, 1, -1).astype(np.int32)

    def score(self, X: np.ndarray, y: np.ndarray) -> float:
        """Accuracy with the cascade's s >= 0 rule; the HIP backend counts on the device."""
        r, be, y = self.result, self._be, np.asarray(y)
        if be.name == "hip" and len(r.sv) and len(y):
            X = np.ascontiguousarray(X, dtype=np.uint8 if X.dtype == np.uint8 else np.float64)
            Xq = be.to_rows(X, self.device)
            be.scale_(Xq, r.mn, r.mx)
            return be.count_correct(be.decision_device(r.sv.X, r.sv.alpha * r.sv.y, Xq, r.b), y) / len(y)
        return float(np.mean(self.predict(X) == y))

    def save(self, directory) -> None:
        from ..models.model_io import save_model

        r = self.result
        rows = r.sv.X[:, : self._be.d].cpu().numpy()
        from ..utils.data import MinMaxScaler

        save_model(directory, r.sv.ids, r.sv.y, r.sv.alpha, r.b, sv_rows=rows,
                   scaler=MinMaxScaler(r.mn.cpu().numpy(), r.mx.cpu().numpy()), params=self.params,
                   meta={"topology": self.topology, "rounds": r.rounds, "world": self.t.world,
                         "sv_history": r.sv_history})

    def summary(self) -> dict:
        r = self.result
        return {"topology": self.topology, "world": self.t.world, "rounds": r.rounds, "converged": r.converged,
                "n_sv": len(r.sv), "b": r.b, "train_ms": r.train_ms, "sv_history": r.sv_history,
                "merged_history": r.merged_history, "round_ms": r.round_ms}


def partition_bounds(n_total: int, world: int, rank: int):
    """Contiguous chunks of ceil(N/P) rows (mpi_svm_main3.cpp:464-518)."""
    chunk = (n_total + world - 1) // world
    lo = min(n_total, rank * chunk)
    return lo, min(n_total, lo + chunk)
