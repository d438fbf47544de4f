#!/usr/bin/env python3
"""One decomposition fit with the inner-kernel shape from the environment (SVM355_DECOMP_NT,
SVM355_DECOMP_PROF=1 prints clock64 ticks per pair update and phase): the working-set size from argv.

    SVM355_DECOMP_PROF=1 SVM355_DECOMP_NT=65 python scripts/decomp_inner_probe.py 60000 384
"""
import sys
import time

from svm355 import SVC
from svm355.utils.data import synthetic_mnist

n, q = int(sys.argv[1]), int(sys.argv[2])
tr = synthetic_mnist(n, seed=2024).compact()
SVC(device="cuda:0", working_set=q).fit(tr.X, tr.y)  # warm
t0 = time.perf_counter()
m = SVC(device="cuda:0", working_set=q).fit(tr.X, tr.y)
dt = (time.perf_counter() - t0) * 1e3
t = m.timings_
print(f"n={n} q={q}: fit {dt:.2f} ms smo {t['smo_ms']:.2f} ms outer {t['outer_iterations']} inner "
      f"{t['inner_iterations']} b {m.b_:.10f} nsv {len(m.support_)}", flush=True)
