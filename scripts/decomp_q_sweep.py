#!/usr/bin/env python3
"""Decomposition fit time per working-set size q (best of 3 after a warm-up), sizes and q values from
argv: python scripts/decomp_q_sweep.py 60000,120000 512,768,1024"""
import sys
import time

from svm355 import SVC
from svm355.utils.data import synthetic_mnist

for n in (int(v) for v in sys.argv[1].split(",")):
    tr = synthetic_mnist(n, seed=2024).compact()
    for q in (int(v) for v in sys.argv[2].split(",")):
        SVC(device="cuda:0", working_set=q).fit(tr.X, tr.y)
        best = 1e30
        for _ in range(3):
            t0 = time.perf_counter()
            m = SVC(device="cuda:0", working_set=q).fit(tr.X, tr.y)
            best = min(best, time.perf_counter() - t0)
        t = m.timings_
        print(f"n={n} q={q}: fit {best * 1e3:.2f} ms outer {t['outer_iterations']} pair updates "
              f"{t['inner_iterations']} b {m.b_:.10f} nsv {len(m.support_)}", flush=True)
