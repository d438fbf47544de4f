"""All-digit one-vs-rest at 60k, batched solver: first-order (default) vs the opt-in second-order selection;
per-class iterations and fit times (best of 2 after a warm-up fit each)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import OneVsRestSVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

tr = synthetic_mnist(60000, seed=2024).compact()
te = synthetic_mnist(10000, seed=2024, offset=60000).compact()
for wss in ("first", "second"):
    OneVsRestSVC(device="cuda:0", wss=wss).fit(tr.X, tr.labels)
    best, m = 1e9, None
    for _ in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        m = OneVsRestSVC(device="cuda:0", wss=wss).fit(tr.X, tr.labels)
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) * 1e3)
    print(f"wss={wss:6s} fit best {best:.1f} ms  smo {m.timings_['smo_ms_all_classes']:.1f} ms  solver {m.timings_['smo_solver']}  "
          f"iterations {m.n_iter_.tolist()} sum {int(m.n_iter_.sum())}  accuracy {m.score(te.X, te.labels):.4f}", flush=True)
