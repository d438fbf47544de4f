#!/usr/bin/env python3
"""One-vs-rest decomposition fits at 60k with 3 / 5 / 10 concurrent class solves (4 warm fits each)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from svm355 import OneVsRestSVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

tr = synthetic_mnist(60000, seed=2024).compact()
OneVsRestSVC(device="cuda:0", solver="decomp").fit(tr.X, tr.labels)  # contexts of the pool threads
for w in (10, 5, 3, 10):
    ts = []
    for _ in range(4):
        torch.cuda.synchronize()
        t = time.perf_counter()
        m = OneVsRestSVC(device="cuda:0", solver="decomp", concurrent_solves=w).fit(tr.X, tr.labels)
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t))
    print(f"workers {w:2d}: {['%.1f' % x for x in ts]} ms  median {np.median(ts):.1f}", flush=True)
