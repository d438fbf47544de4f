"""Two 60k SVC fits (upload, scaling, exact-integer Gram, persistent SMO) -- a short program for
rocprofv3 counter passes over the headline kernels."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
tr = synthetic_mnist(n, seed=2024).compact()
for _ in range(2):
    m = SVC(device="cuda:0").fit(tr.X, tr.y)
torch.cuda.synchronize()
print(f"done: {m.n_iter_} iterations, b={m.b_:.12f}", flush=True)
