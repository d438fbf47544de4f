"""Cascade SVM (classical tree, mpi_svm_main3.cpp; modified two-layer star, mpi_svm_main2.cpp):
a binding of the ONE native driver in ``csrc/cascade`` (round logic, warm starts, ID de-duplication,
ID-set convergence, checkpoint/resume, abort on failure).

* ``fit(X, y, world=P)`` on ``device="cpu"``: P thread-ranks on the C++ oracle backend (loopback
  transport) — the test vehicle of the exact code the GPUs run.
* ``fit(X, y, world=P)`` on ``device="cuda"``: P thread-ranks on P GPUs of this process
  (``DeviceGroup``: ncclCommInitAll, RCCL over xGMI) or a loopback rehearsal on fewer GPUs.
* ``fit_rank(rank, X_part, y_part, ids, n_total)``: one rank per process (``RcclRank``, e.g. under
  torchrun; ``HostCommRank``: the same on the CPU oracle over a gloo group).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .. import _native as N
from ..utils.config import SVMParams
from ..utils.trace import trace_range

LAYER_NAMES = {0: "local", -1: "merge"}
SOLVER_NAMES = {0: "smo", 1: "decomp"}


@dataclass
class CascadeResult:
    ids: np.ndarray  # final global SV ids
    y: np.ndarray
    alpha: np.ndarray
    sv_rows: np.ndarray  # scaled SV rows (n_sv x d)
    mn: np.ndarray
    mx: np.ndarray
    b: float
    rounds: int
    converged: bool
    train_ms: float  # max over the ranks this call drove
    world: int
    transport: str
    backend: str
    sv_history: List[int] = field(default_factory=list)
    merged_history: List[int] = field(default_factory=list)
    round_ms: List[float] = field(default_factory=list)
    rank_train_ms: List[float] = field(default_factory=list)
    solves: List[dict] = field(default_factory=list)
    phase_ms: dict = field(default_factory=dict)  # lowest driven rank, per driver phase

    @classmethod
    def take(cls, p) -> "CascadeResult":
        """Copy a native svm_cascade_out and free it."""
        if not p:
            raise N.NativeError(N.last_error())
        o = p.contents
        try:
            arr = lambda ptr, n, dt: np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt, copy=True) if n else np.empty(0, dt)
            sol = arr(o.solves, N.SOLVE_COLS * o.n_solves, np.float64).reshape(-1, N.SOLVE_COLS)
            solves = [{"rank": int(s[0]), "round": int(s[1]),
                       "layer": LAYER_NAMES.get(int(s[2]), f"layer{int(s[2])}"), "n": int(s[3]),
                       "iterations": int(s[4]), "ms": float(s[5]), "b": float(s[6]),
                       "stop": N.STOP_NAMES.get(int(s[7]), str(int(s[7]))), "gram_ms": float(s[8]), "skipped": bool(s[9]),
                       "row_cache": bool(s[10]), "solo_ms": float(s[11]),
                       "solver": SOLVER_NAMES.get(int(s[12]), str(int(s[12]))), "outer": int(s[13])} for s in sol]
            phases = dict(zip(N.CASCADE_PHASES, [round(float(v), 3) for v in o.phase_ms]))
            return cls(arr(o.ids, o.n_sv, np.int64), arr(o.y, o.n_sv, np.int32), arr(o.alpha, o.n_sv, np.float64),
                       arr(o.sv_rows, o.n_sv * o.d, np.float64).reshape(o.n_sv, o.d), arr(o.mn, o.d, np.float64),
                       arr(o.mx, o.d, np.float64), float(o.b), int(o.rounds), bool(o.converged), float(o.train_ms),
                       int(o.world), o.transport.decode(), o.backend.decode(),
                       arr(o.sv_history, o.n_hist, np.int64).tolist(), arr(o.merged_history, o.n_merged, np.int64).tolist(),
                       arr(o.round_ms, o.n_hist, np.float64).tolist(), arr(o.rank_train_ms, o.n_ranks, np.float64).tolist(),
                       solves, phases)
        finally:
            N.core().svm_cascade_free(p)


class CascadeSVM:
    def __init__(self, params: Optional[SVMParams] = None, topology: str = "star", max_rounds: int = 50,
                 checkpoint_dir: Optional[str] = None, resume: bool = False, verbose: int = 0,
                 comm_timeout_s: float = 600.0, fail_rank: int = -1, fail_round: int = -1,
                 fail_stall_s: float = 0.0, solver: str = "auto"):
        if topology not in ("star", "tree"):
            raise ValueError("topology must be 'star' (modified two-layer) or 'tree' (classical)")
        if solver not in ("auto", "smo", "decomp"):
            raise ValueError("solver must be 'auto' (GPUs: per solve, the decomposition for cold / small sets and "
                             "the pairwise SMO for large warm ones; CPU: the pairwise oracle), 'smo' (the reference's "
                             "pairwise trajectory) or 'decomp' (the warm-started working-set decomposition)")
        # every local / merge solve: the warm-started working-set decomposition (decomp.hip; on the CPU
        # backend its oracle on the set's kernel matrix), the reference's pairwise SMO, or per solve
        self.solver = solver
        self.params = params or SVMParams()
        self.topology = topology
        self._ck = checkpoint_dir.encode() if checkpoint_dir else None  # kept alive for the C struct
        self.cfg = N.SvmCascadeCfg()
        N.core().svm_cascade_default_cfg(ctypes.byref(self.cfg))
        c = self.cfg
        c.tree, c.max_rounds, c.params, c.log = int(topology == "tree"), max_rounds, self.params.to_struct(), int(verbose > 0)
        c.resume, c.checkpoint_dir, c.comm_timeout_s = int(resume), self._ck, comm_timeout_s
        c.fail_rank, c.fail_round, c.fail_stall_s = fail_rank, fail_round, fail_stall_s
        self.result: Optional[CascadeResult] = None
        self.device = "cpu"

    def _set_solver(self, cpu: bool) -> None:
        # auto on GPUs: per solve (svm_cascade_cfg.solver = 2) -- the decomposition for cold and small
        # sets, the pairwise SMO for large warm-started ones (cascade.h cascade_solver_for)
        s = self.solver if self.solver != "auto" else ("smo" if cpu else "per-solve")
        self.cfg.solver = {"smo": 0, "decomp": 1, "per-solve": 2}[s]
        self.solver_used = s

    def _check_world(self, world: int) -> None:
        if self.topology == "tree" and world & (world - 1):  # mpi_svm_main3.cpp:420-428
            raise ValueError(f"classical (tree) cascade needs a power-of-2 number of ranks, got {world}")

    def fit(self, X, y, world: int = 1, device: str = "cpu", transport: str = "auto", group=None) -> "CascadeSVM":
        """Thread-ranks of this process over contiguous ceil(n / world) partitions with global ids."""
        self._check_world(world)
        self._set_solver(device == "cpu")
        y = np.ascontiguousarray(y, dtype=np.int32)
        if device == "cpu":
            X = np.ascontiguousarray(X, dtype=np.float64)
            p = N.core().svm_cascade_fit_cpu(N.ptr(X), N.ptr(y), X.shape[0], X.shape[1], world, ctypes.byref(self.cfg))
        else:
            from .rccl import DeviceGroup

            X = np.ascontiguousarray(X, dtype=np.uint8 if X.dtype == np.uint8 else np.float64)
            g = group or DeviceGroup.shared(world, transport)
            with trace_range(f"svm355.cascade.{self.topology} world={world} solver={self.solver_used}"):
                p = N.hip().svmd_cascade_group_fit(g.handle, N.ptr(X), int(X.dtype == np.uint8), N.ptr(y),
                                                   X.shape[0], X.shape[1], ctypes.byref(self.cfg))
            if not p:
                err = N.last_error()
                if group is None and g.broken:  # aborted communicators: the next fit builds a new group
                    DeviceGroup._shared.pop((world, transport), None)
                    g.close()
                raise N.NativeError(err)
        self.device = device
        self.result = CascadeResult.take(p)
        return self

    def fit_rank(self, rank, X_part, y_part, ids, n_total: int) -> "CascadeSVM":
        """This process's rank trains on its partition (raw rows, global ids): ``RcclRank`` (its GPU,
        RCCL) or ``HostCommRank`` (the CPU oracle over a gloo group, the multi-process CPU tests)."""
        self._check_world(rank.world)
        self._set_solver(rank.device == "cpu")
        if rank.device == "cpu":
            self.device = "cpu"
            self.result = CascadeResult.take(rank.fit(self.cfg, X_part, y_part, ids, n_total))
            return self
        X = np.ascontiguousarray(X_part, dtype=np.uint8 if X_part.dtype == np.uint8 else np.float64)
        y = np.ascontiguousarray(y_part, dtype=np.int32)
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        p = N.hip().svmd_cascade_rank_fit(rank.handle, N.ptr(X), int(X.dtype == np.uint8), N.ptr(y), N.ptr(ids),
                                          X.shape[0], X.shape[1], int(n_total), ctypes.byref(self.cfg))
        self.device = f"cuda:{rank.device}"
        self.result = CascadeResult.take(p)
        return self

    # ---- inference over the final SVs (decision = sum alpha y K - b; the cascades map s >= 0 to +1)
    def _model(self):
        from ..models.svc import SVC
        from ..utils.data import MinMaxScaler

        r, p = self.result, self.params
        m = SVC(C=p.C, gamma=p.gamma, tol=p.tau, eps=p.eps, sv_tol=p.sv_tol, max_iter=p.max_iter,
                device=self.device, zero_is_positive=True)
        m.scaler_, m.support_, m.support_labels_ = MinMaxScaler(r.mn, r.mx), r.ids, r.y
        m.b_, m.intercept_, m.support_vectors_, m.dual_coef_ = r.b, -r.b, r.sv_rows, r.alpha * r.y
        m.alpha_ = np.zeros(int(r.ids.max()) + 1 if len(r.ids) else 0)
        m.alpha_[r.ids] = r.alpha
        if self.device != "cpu":
            m._upload_model(self.device)
        return m

    def decision_function(self, X) -> np.ndarray:
        return self._model().decision_function(X)

    def predict(self, X) -> np.ndarray:
        return self._model().predict(X)

    def score(self, X, y) -> float:
        return self._model().score(X, y)

    def save(self, directory) -> None:
        """Reference model files (final_sv_{ids,labels,alphas}.txt, final_b.txt, M3 :754-770) + extras."""
        from ..models.model_io import save_model
        from ..utils.data import MinMaxScaler

        r = self.result
        save_model(directory, ids=r.ids, labels=r.y, alphas=r.alpha, b=r.b, sv_rows=r.sv_rows,
                   scaler=MinMaxScaler(r.mn, r.mx), params=self.params,
                   meta={"topology": self.topology, "rounds": r.rounds, "world": r.world, "sv_history": r.sv_history})

    def summary(self) -> dict:
        r = self.result
        return {"topology": self.topology, "world": r.world, "rounds": r.rounds, "converged": r.converged,
                "n_sv": len(r.ids), "b": r.b, "train_ms": r.train_ms, "sv_history": r.sv_history,
                "merged_history": r.merged_history, "round_ms": r.round_ms, "transport": r.transport,
                "backend": r.backend}


def partition_bounds(n_total: int, world: int, rank: int):
    """Contiguous chunks of ceil(N/P) rows (mpi_svm_main3.cpp:464-518)."""
    chunk = (n_total + world - 1) // world
    lo = min(n_total, rank * chunk)
    return lo, min(n_total, lo + chunk)


def critical_path(solves, topology: str):
    """Per round: the slowest rank's local solve (tree: slowest rank of the first layer) + rank 0's
    merge (tree: slowest rank of every later layer), i.e. the solve time of a run with one GPU per
    rank, exchanges excluded.  Solve times are the solo device times when the run measured them
    (SVM355_CASCADE_SERIAL_SOLVES=1: ranks sharing one GPU take turns, so each solve is timed as on a
    GPU of its own), else wall times.  ``solves`` = ``CascadeResult.solves`` of every rank.
    Returns ([[round, local_max_ms, merge_ms, local_max_iterations, merge_iterations]], total ms)."""
    solves = [dict(s, ms=s["solo_ms"]) if s.get("solo_ms", -1.0) >= 0 else s for s in solves]
    out, tot = [], 0.0
    for r in sorted({s["round"] for s in solves}):
        rs = [s for s in solves if s["round"] == r]
        if topology == "star":
            loc = [s for s in rs if s["layer"] == "local"]
            mer = [s for s in rs if s["layer"] == "merge"]
            lm = max((s["ms"] for s in loc), default=0.0)
            li = max((s["iterations"] for s in loc), default=0)
            mm = sum(s["ms"] for s in mer)
            mi = sum(s["iterations"] for s in mer)
        else:
            layers = sorted({s["layer"] for s in rs}, key=lambda x: int(x[5:]))
            first = [s for s in rs if s["layer"] == layers[0]] if layers else []
            lm = max((s["ms"] for s in first), default=0.0)
            li = max((s["iterations"] for s in first), default=0)
            mm = sum(max(s["ms"] for s in rs if s["layer"] == L) for L in layers[1:])
            mi = sum(max(s["iterations"] for s in rs if s["layer"] == L) for L in layers[1:])
        out.append([r, round(lm, 3), round(mm, 3), li, mi])
        tot += lm + mm
    return out, round(tot, 3)



def loopback_exercise(world: int, script: str, strict: bool = True, timeout_s: float = 20.0):
    """Run a transport call script (csrc/cascade/exercise.cpp syntax) on ``world`` CPU thread-ranks
    over the loopback transport, every received byte checked.  Returns the elapsed seconds; raises
    ``NativeError`` naming the ranks / op on a mismatch, deadlock, wrong payload or timeout."""
    el = ctypes.c_double(0.0)
    rc = N.core().svm_loopback_exercise(int(world), script.encode(), int(bool(strict)), float(timeout_s),
                                         ctypes.byref(el))
    if rc != 0:
        raise N.NativeError(f"{N.last_error()} (after {el.value:.2f} s)")
    return el.value


def preflight_script(world: int, bulk_bytes: int = 1 << 20) -> str:
    """The op list the device groups / ranks run on their RCCL communicators before any fit."""
    lib = N.core()
    need = lib.svm_preflight_script(int(world), int(bulk_bytes), None, 0)
    buf = ctypes.create_string_buffer(need)
    N.check(lib.svm_preflight_script(int(world), int(bulk_bytes), buf, need), "svm_preflight_script")
    return buf.value.decode()
