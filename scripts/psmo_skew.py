"""Exchange-skew diagnostic of the persistent SMO (SVM355_PSMO_STAMP=2): per-phase cycles, the spread
of the workgroups' record publications and workgroup 0's wait past the last one, per solver mode.

    python scripts/psmo_skew.py [n]
"""
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
mn, mx, sqn = D.minmax_scale_(Xd, 784)
K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
yd = torch.from_numpy(tr.y).to(dev)
os.environ["SVM355_SMO"] = "persistent"
os.environ["SVM355_PSMO_STAMP"] = "2"
for xcd in ("0", "1"):
    os.environ["SVM355_PSMO_XCD"] = xcd
    print(f"--- n={n} xcd-local={xcd}", file=sys.stderr, flush=True)
    a = torch.zeros(n, dtype=torch.float64, device=dev)
    r, _ = D.smo(K, yd, a, SVMParams(), n=n)
    torch.cuda.synchronize()
    print(f"n={n} xcd={xcd}: iterations {r.iterations} b {r.b:.15f}", flush=True)
