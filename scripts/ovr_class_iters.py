"""Per-class SMO iteration counts of the all-digit one-vs-rest fit at 60k (load balance of the
batched XCD-team solver: 10 classes on 8 teams)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import OneVsRestSVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

tr = synthetic_mnist(60000, seed=2024).compact()
m = OneVsRestSVC(device="cuda:0").fit(tr.X, tr.labels)
for _ in range(2):
    torch.cuda.synchronize()
    t = time.perf_counter()
    m = OneVsRestSVC(device="cuda:0").fit(tr.X, tr.labels)
    torch.cuda.synchronize()
    print("fit ms", round((time.perf_counter() - t) * 1e3, 1), m.timings_, flush=True)
print("iterations per class", m.n_iter_.tolist(), "sum", int(m.n_iter_.sum()), flush=True)
