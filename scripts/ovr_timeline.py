#!/usr/bin/env python3
"""One-vs-rest decomposition at 60k: every class alone (concurrent_solves=1, per-class time from the fit's
timings) and all ten at once, for a kernel-trace timeline (scripts/rocpd_timeline.py)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from svm355 import OneVsRestSVC, SVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

tr = synthetic_mnist(60000, seed=2024).compact()
OneVsRestSVC(device="cuda:0", solver="decomp").fit(tr.X, tr.labels)  # pool threads' contexts
per = []
for c in range(10):
    y = np.where(tr.labels == c, 1, -1).astype(np.int32)
    SVC(device="cuda:0", solver="decomp").fit(tr.X, y)
    torch.cuda.synchronize()
    t = time.perf_counter()
    m = SVC(device="cuda:0", solver="decomp").fit(tr.X, y)
    torch.cuda.synchronize()
    per.append(1e3 * (time.perf_counter() - t))
    print(f"class {c}: {per[-1]:.2f} ms outer {m.timings_['outer_iterations']} pairs {m.timings_['inner_iterations']}", flush=True)
print(f"sum {sum(per):.1f} ms, max {max(per):.1f} ms", flush=True)
for k in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    OneVsRestSVC(device="cuda:0", solver="decomp").fit(tr.X, tr.labels)
    torch.cuda.synchronize()
    print(f"ovr concurrent fit {k}: {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
