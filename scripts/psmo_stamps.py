"""Diagnostic: per-phase cycle breakdown of the persistent SMO (s_memtime stamps build)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
dev = torch.device("cuda:0")
tr = synthetic_mnist(n, seed=2024)
Xd = D.upload_rows(tr.X, dev)
_, _, sqn = D.minmax_scale_(Xd, 784)
K = D.rbf_gram(Xd, sqn, Xd, sqn, 0.00125, symmetric=True)
yd = torch.from_numpy(tr.y).to(dev)
os.environ["SVM355_SMO"] = "persistent"
os.environ["SVM355_PSMO_STAMP"] = "1"
for wg in sys.argv[2:] or ["32", "64", "128"]:
    os.environ["SVM355_PSMO_WG"] = wg
    a = torch.zeros(n, dtype=torch.float64, device=dev)
    r, _ = D.smo(K, yd, a, SVMParams(), n=n)
    torch.cuda.synchronize()
    print(f"G<={wg}: iterations {r.iterations} {r.seconds*1e3:.1f} ms", flush=True)
