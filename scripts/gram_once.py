"""Two exact-integer Gram evaluations at n (default 60k) -- a short program for rocprofv3 passes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
dev = torch.device("cuda:0")
tr = synthetic_mnist(n, seed=2024)
Xd = D.upload_rows(tr.X, dev)
mn, mx, sqn = D.minmax_scale_(Xd, 784)
K = torch.empty((n, (n + 1) // 2 * 2), dtype=torch.float64, device=dev)
for _ in range(2):
    D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, gram="int", out=K)
torch.cuda.synchronize()
print("done", flush=True)
