"""Time the RBF Gram kernel variants on one device (interleaved rounds, same process)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355.ops import device as D  # noqa: E402
from svm355.ops import cpu as C  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402
import numpy as np  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
dev = torch.device("cuda:0")
tr = synthetic_mnist(n, seed=2024)
Xd = D.upload_rows(tr.X, dev)
_, _, sqn = D.minmax_scale_(Xd, 784)
K = torch.empty((n, (n + 1) // 2 * 2), dtype=torch.float64, device=dev)
res = {}
for rnd in range(3):
    for tri in ("1", "0"):
        os.environ["SVM355_GRAM_TRI"] = tri
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.rbf_gram(Xd, sqn, Xd, sqn, 0.00125, symmetric=True, out=K)
        torch.cuda.synchronize()
        res.setdefault(tri, []).append((time.perf_counter() - t0) * 1e3)
flop = 2.0 * n * n * 784
for tri, v in res.items():
    best = min(v)
    eff = flop / (2 if tri == "1" else 1)
    print(f"tri={tri}: min {best:.2f} ms  median {sorted(v)[1]:.2f} ms  -> {eff / best / 1e9:.1f} TFLOP/s executed, "
          f"{flop / best / 1e9:.1f} TFLOP/s full-Gram-equivalent", flush=True)
# correctness spot check of the triangular variant against the CPU reference on a few rows
os.environ["SVM355_GRAM_TRI"] = "1"
D.rbf_gram(Xd, sqn, Xd, sqn, 0.00125, symmetric=True, out=K)
rows = np.array([0, 1, 127, 128, n // 2, n - 1])
Xs = Xd[:, :784].cpu().numpy()
ref = C.rbf_matrix(Xs[rows], Xs, 0.00125, 16)
got = K[torch.from_numpy(rows).to(dev), :n].cpu().numpy()
print("max |K - ref| on sample rows:", float(np.abs(got - ref).max()), " symmetric:",
      bool(torch.equal(K[:2000, :2000], K[:2000, :2000].T)))
