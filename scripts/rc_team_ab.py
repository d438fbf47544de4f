"""A/B of the persistent row-cache solver's team width (SVM355_RC_MAXG = 64 / 128 / 256) in ONE
process: the data, the quantised rows and the cache allocation are warm, caps alternate, best of R."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
reps = int(os.environ.get("REPS", "2"))
for n in [int(x) for x in (sys.argv[1:] or ["250000"])]:
    tr = synthetic_mnist(n, seed=2024).compact()
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    yd = torch.from_numpy(tr.y).to(dev)
    best = {}
    for rep in range(reps + 1):  # rep 0 warms everything up
        for cap in os.environ.get("CAPS", "64,128,256").split(","):
            os.environ["SVM355_RC_MAXG"] = cap
            a = torch.zeros(n, dtype=torch.float64, device=dev)
            torch.cuda.synchronize()
            t = time.perf_counter()
            r, tm = D.train(Xd, sqn, yd, a, SVMParams(), mn=mn, mx=mx, kcache="rows")
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) * 1e3
            if rep:
                best[cap] = min(best.get(cap, 1e18), ms)
            print(f"n={n} cap={cap} rep={rep}: {ms:.0f} ms, iters {r.iterations}, b {r.b!r}", flush=True)
    print(f"n={n} best: " + " | ".join(f"cap {c}: {v:.0f} ms" for c, v in best.items()), flush=True)
