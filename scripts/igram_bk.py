"""Gram-only timing of the exact-integer kernel at the two LDS stage depths (SVM355_IGRAM_BK)."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
for n in (7500, 60000):
    tr = synthetic_mnist(n, seed=2024)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K = torch.empty((n, (n + 1) // 2 * 2), dtype=torch.float64, device=dev)
    ref = None
    for bk in ("64", "128", "64", "128"):
        os.environ["SVM355_IGRAM_BK"] = bk
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, gram="int", out=K)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        chk = K[:500, :n].clone()
        ref = chk if ref is None else ref
        print(f"n={n} BK={bk}: {best * 1e3:.2f} ms  identical={bool(torch.equal(chk, ref))}", flush=True)
