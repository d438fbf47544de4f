"""Persistent-SMO launch shape vs n: device-wide (64 WGs x 512) vs XCD-local (one XCD's L2 exchange)
at 512 and 1024 threads per workgroup.  The SMO launcher reads SVM355_PSMO_* per call, so one
process times every variant on the same resident Gram; models must be identical.

    python scripts/smo_shape_sweep.py [n1,n2,...]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

VARIANTS = {
    "device-wide NT=512": {"SVM355_PSMO_XCD": "0", "SVM355_PSMO_NT": "512"},
    "xcd NT=1024": {"SVM355_PSMO_XCD": "1", "SVM355_PSMO_NT": "1024", "SVM355_PSMO_LDS": "0"},
    "xcd NT=512": {"SVM355_PSMO_XCD": "1", "SVM355_PSMO_NT": "512", "SVM355_PSMO_LDS": "0"},
    "xcd NT=512 1/CU": {"SVM355_PSMO_XCD": "1", "SVM355_PSMO_NT": "512", "SVM355_PSMO_LDS": "98304"},
    "xcd NT=256": {"SVM355_PSMO_XCD": "1", "SVM355_PSMO_NT": "256", "SVM355_PSMO_LDS": "0"},
    "xcd NT=256 1/CU": {"SVM355_PSMO_XCD": "1", "SVM355_PSMO_NT": "256", "SVM355_PSMO_LDS": "98304"},
    "default": {},
}
if os.environ.get("SHAPE_QUICK"):
    VARIANTS = {k: VARIANTS[k] for k in ("device-wide NT=512", "default")}
KNOBS = ("SVM355_PSMO_XCD", "SVM355_PSMO_NT", "SVM355_PSMO_LDS")
sizes = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "16000,24000,30000,40000,50000,60000").split(",")]
dev = torch.device("cuda:0")
p = SVMParams()
for n in sizes:
    tr = synthetic_mnist(n, seed=2024).compact()
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, tr.X.shape[1])
    K, _ = D.rbf_gram_sym(Xd, sqn, p.gamma, mn=mn, mx=mx)
    y = torch.from_numpy(tr.y).to(dev)
    ref = None
    for name, env in VARIANTS.items():
        for k in KNOBS:
            os.environ.pop(k, None)
        os.environ.update(env)
        ts = []
        for rep in range(4):
            a = torch.zeros(n, dtype=torch.float64, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r, _ = D.smo(K, y, a, p)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        sig = (r.iterations, r.b)
        ref = ref or sig
        best = min(ts[1:])
        print(f"n={n:6d} {name:18s} smo {best:7.2f} ms  {best * 1e3 / r.iterations:6.3f} us/iter  "
              f"iters {r.iterations}  identical={sig == ref}", flush=True)
    for k in KNOBS:
        os.environ.pop(k, None)
    del K
