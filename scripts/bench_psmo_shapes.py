"""A/B persistent-SMO grid shapes (threads per workgroup NT x workgroups G) on one resident Gram.

Every shape must reproduce the same trajectory (iterations, b); reports the best of 3 runs."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
shapes = [tuple(int(v) for v in s.split("x")) for s in (sys.argv[2:] or ["256x64", "512x64", "1024x64", "512x32"])]
dev = torch.device("cuda:0")
tr = synthetic_mnist(n, seed=2024)
Xd = D.upload_rows(tr.X, dev)
mn, mx, sqn = D.minmax_scale_(Xd, 784)
K, path = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
yd = torch.from_numpy(tr.y).to(dev)
os.environ["SVM355_SMO"] = "persistent"
res = {s: [] for s in shapes}
for rnd in range(3):
    for nt, wg in shapes:
        os.environ["SVM355_PSMO_NT"] = str(nt)
        os.environ["SVM355_PSMO_WG"] = str(wg)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r, _ = D.smo(K, yd, a, SVMParams(), n=n)
        torch.cuda.synchronize()
        res[(nt, wg)].append(((time.perf_counter() - t0) * 1e3, r.iterations, r.b))
ref = None
for s, v in res.items():
    best = min(x[0] for x in v)
    it, b = v[0][1], v[0][2]
    ref = ref or (it, b)
    same = (it, b) == ref
    print(f"NT={s[0]:4d} G<={s[1]:3d}: best {best:7.2f} ms  iters {it}  us/iter {best * 1e3 / it:.3f}  "
          f"b {b:.15f} {'' if same else 'TRAJECTORY DIFFERS'}", flush=True)
if len(sys.argv) > 1 and os.environ.get("PSMO_STAMPS"):
    os.environ["SVM355_PSMO_STAMP"] = "1"
    for nt, wg in shapes:
        os.environ["SVM355_PSMO_NT"] = str(nt)
        os.environ["SVM355_PSMO_WG"] = str(wg)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        D.smo(K, yd, a, SVMParams(), n=n)
        torch.cuda.synchronize()
