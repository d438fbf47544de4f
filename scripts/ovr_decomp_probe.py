#!/usr/bin/env python3
"""One-vs-rest over all ten digits, 60k synthetic MNIST: the batched pairwise solve over the shared Gram
against the decomposition solver per class (no Gram), fit times (warm), per-class iterations, b and SV
counts, test accuracy and prediction agreement."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from svm355 import OneVsRestSVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
tr, te = synthetic_mnist(n, seed=2024).compact(), synthetic_mnist(10000, seed=2024, offset=n).compact()
res = {}
for solver in ("batched", "decomp"):
    ts, m = [], None
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        m = OneVsRestSVC(device="cuda:0", solver=solver).fit(tr.X, tr.labels)
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t))
    acc = m.score(te.X, te.labels)
    res[solver] = m
    nsv = [int(np.count_nonzero(m.dual_coef_[:, c])) for c in range(len(m.classes_))]
    print(f"{solver:8s}: fit {['%.1f' % x for x in ts]} ms  timings {m.timings_}", flush=True)
    print(f"          iterations {m.n_iter_.tolist()}", flush=True)
    print(f"          SVs per class {nsv}  union {len(m.support_)}  accuracy {acc:.4f}", flush=True)
    print(f"          b {[round(float(b), 6) for b in m.intercepts_b_]}", flush=True)
    if solver == "decomp":
        ct = m.class_timings_
        print("          per-class solve ms " + str({k: round(v['smo_ms'], 1) for k, v in ct.items()}), flush=True)
        print("          per-class outer " + str({k: v['outer_iterations'] for k, v in ct.items()}), flush=True)
pa, pb = res["batched"].predict(te.X), res["decomp"].predict(te.X)
print(f"prediction agreement batched vs decomp: {float(np.mean(pa == pb)):.4f}; max |b diff| "
      f"{float(np.max(np.abs(res['batched'].intercepts_b_ - res['decomp'].intercepts_b_))):.2e}", flush=True)
