"""Solver hyper-parameters (the reference's compile-time constants).

| knob      | default  | reference site                                   |
|-----------|----------|--------------------------------------------------|
| C         | 10.0     | main3.cpp:163,342; gpu_svm_main3.cu:319,601      |
| gamma     | 0.00125  | main3.cpp:95 (hard-coded inside kernel())        |
| tau       | 1e-5     | main3.cpp:196,213 (stop: b_low <= b_high + 2 tau)|
| eps       | 1e-12    | main3.cpp:109,128,165 (set membership, eta floor)|
| sv_tol    | 1e-8     | main3.cpp:297,367 (alpha > sv_tol is an SV)      |
| max_iter  | 100000   | main3.cpp:197-198 (num_iter starts at 1)         |
| max_rounds| 50       | mpi_svm_main3.cpp:544, mpi_svm_main2.cpp:428     |
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass

import numpy as np

from .._native import params_struct


def default_threads(cap: int = 16) -> int:
    """CPU workers for the native oracle: the CPUs this process may run on, capped at ``cap``.

    ``os.cpu_count()`` reports the whole machine (hundreds of CPUs on a GPU node) even when the
    process is confined to a few; the O(n) SMO passes gain nothing past ~16 workers."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(cap, n))


@dataclass
class SVMParams:
    C: float = 10.0
    gamma: float = 0.00125
    tau: float = 1e-5
    eps: float = 1e-12
    sv_tol: float = 1e-8
    max_iter: int = 100000
    n_threads: int = 1
    # working-set selection: 1 = first order (the reference, Keerthi et al.), 2 = second-order choice
    # of the second index (Fan, Chen & Lin 2005; opt-in, not the reference's trajectory)
    wss: int = 1
    # shrinking (an active set) in the working-set decomposition solver (decomp_shrink.h): True = on
    # (every 2 outer iterations), False = off (the default: measured slower on the headline shapes), an
    # int k > 0 = a pass every k outer iterations.  The stop test is still the reference's, on all n
    # points (f recomputed when the solve unshrinks).
    shrinking: object = False

    def __post_init__(self):
        # the reference hard-codes these; as parameters they must keep the problem well posed:
        # C <= 0 empties the box, gamma <= 0 makes the kernel constant (eta = 0), tau <= 0 never stops
        bad = [f"{k}={v!r}" for k, v, ok in (("C", self.C, self.C > 0), ("gamma", self.gamma, self.gamma > 0),
                                              ("tau", self.tau, self.tau > 0), ("eps", self.eps, self.eps >= 0),
                                              ("sv_tol", self.sv_tol, self.sv_tol >= 0),
                                              ("max_iter", self.max_iter, self.max_iter >= 1),
                                              ("n_threads", self.n_threads, self.n_threads >= 0),
                                              ("wss", self.wss, self.wss in (1, 2)),
                                              ("shrinking", self._shrink_code(), self._shrink_code() >= -1))
               if not (ok and np.isfinite(v))]
        if bad:
            raise ValueError("SVM parameters out of range: " + ", ".join(bad) +
                             " (C, gamma, tau > 0; eps, sv_tol >= 0; max_iter >= 1; wss 1 or 2)")

    def _shrink_code(self) -> int:
        s = self.shrinking
        if isinstance(s, (bool, np.bool_)):
            return 2 if s else 0
        try:
            k = int(s)
        except (TypeError, ValueError):
            return -2
        return k if k >= 0 and k == s else -2  # 0: off, k > 0: a pass every k outer iterations

    def to_struct(self, verbose: int = 0):
        return params_struct(self.C, self.gamma, self.tau, self.eps, self.sv_tol, self.max_iter,
                             self.n_threads, verbose, self.wss, self._shrink_code())

    def replace(self, **kw) -> "SVMParams":
        return dataclasses.replace(self, **kw)

    def as_dict(self) -> dict:
        return dataclasses.asdict(self)
