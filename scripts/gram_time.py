"""Exact-integer Gram time at n (best of R), for A/B builds via SVM355_LIB_DIR."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
tr = synthetic_mnist(n, seed=2024)
Xd = D.upload_rows(tr.compact().X, dev)
mn, mx, sqn = D.minmax_scale_(Xd, 784)
K = None
best = 1e9
for _ in range(6):
    torch.cuda.synchronize()
    t = time.perf_counter()
    K, info = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, out=K)
    torch.cuda.synchronize()
    best = min(best, time.perf_counter() - t)
print(f"{os.environ.get('TAG', '')} n={n} gram best {best * 1e3:.2f} ms {info}", flush=True)
