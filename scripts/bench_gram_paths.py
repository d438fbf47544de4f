"""Gram-only timing: exact-integer (int8 MFMA) vs FP64 MFMA path at several n (best of 3)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
for n in [int(v) for v in (sys.argv[1:] or ["7500", "30000", "60000"])]:
    tr = synthetic_mnist(n, seed=2024)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K = torch.empty((n, (n + 1) // 2 * 2), dtype=torch.float64, device=dev)
    res = {}
    for g in ("int", "fp64"):
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, gram=g, out=K)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e3)
        res[g] = best
        if g == "int":
            Ki = K[:2000, :n].clone()
    diff = (Ki - K[:2000, :n]).abs().max().item()
    print(f"n={n:6d}: int8-exact {res['int']:8.3f} ms   fp64 {res['fp64']:8.3f} ms   max|dK| (2000 rows) {diff:.2e}",
          flush=True)
