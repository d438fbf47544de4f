"""A/B the device SMO paths on one resident Gram (same process, interleaved rounds)."""
import os
import sys
import time

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
torch.cuda.synchronize()
t0 = time.perf_counter()
K = D.rbf_gram(Xd, sqn, Xd, sqn, 0.00125, symmetric=True)
torch.cuda.synchronize()
print(f"gram {n}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
yd = torch.from_numpy(tr.y).to(dev)
configs = [("graph", None), ("persistent", 32), ("persistent", 64), ("persistent", 128), ("persistent", 256)]
res = {c: [] for c in configs}
for rnd in range(3):
    for mode, wg in configs:
        os.environ["SVM355_SMO"] = mode
        if wg:
            os.environ["SVM355_PSMO_WG"] = str(wg)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r, _ = D.smo(K, yd, a, SVMParams(), n=n)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        res[(mode, wg)].append((dt, r.iterations, r.b))
for c, v in res.items():
    dts = sorted(x[0] for x in v)
    it = v[0][1]
    print(f"{c[0]:>10} G<={c[1]}: median {dts[len(dts)//2]:.2f} ms  min {dts[0]:.2f} ms  iters {it}  "
          f"us/iter {dts[0]*1e3/it:.2f}  b {v[0][2]:.15f}", flush=True)
