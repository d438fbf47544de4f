"""How often does the XCD-local SMO find fewer than G workgroups on XCD 0?  Sequential solves of
one 60k problem for several registration windows (SVM355_PSMO_REG_US); the native library prints
one line per fallback.  Then batched one-vs-rest solves with the per-XCD team report.

    python scripts/xcd_register_probe.py [n] [reps]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
dev = torch.device("cuda:0")
p = SVMParams()
tr = synthetic_mnist(n, seed=2024).compact()
Xd = D.upload_rows(tr.X, dev)
mn, mx, sqn = D.minmax_scale_(Xd, tr.X.shape[1])
K, _ = D.rbf_gram_sym(Xd, sqn, p.gamma, mn=mn, mx=mx)
y = torch.from_numpy(tr.y).to(dev)
for us in ("2000", "20000"):
    os.environ["SVM355_PSMO_REG_US"] = us
    print(f"--- window {us} us, {reps} sequential solves", flush=True)
    ts = []
    for _ in range(reps):
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.smo(K, y, a, p)
        torch.cuda.synchronize()
        ts.append(round((time.perf_counter() - t0) * 1e3, 1))
    print("smo ms:", ts, flush=True)
os.environ.pop("SVM355_PSMO_REG_US")
os.environ["SVM355_SMO_MULTI_DEBUG"] = "1"
Y = torch.stack([torch.from_numpy((tr.labels == c).astype("int32") * 2 - 1) for c in range(10)]).to(dev)
for _ in range(3):
    A = torch.zeros((10, n), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rs, batched = D.smo_multi(K, Y, A, p)
    torch.cuda.synchronize()
    print(f"batched={batched} {(time.perf_counter() - t0) * 1e3:.1f} ms iters {[r.iterations for r in rs]}", flush=True)
