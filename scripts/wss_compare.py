"""First- vs second-order working-set selection on one resident Gram (persistent solver): iterations,
solve time (best of R), #SV, b and test accuracy of the resulting models."""
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from svm355 import SVC, SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
R = int(os.environ.get("REPS", "5"))
for n in [int(x) for x in (sys.argv[1:] or ["60000"])]:
    tr = synthetic_mnist(n, seed=2024)
    te = synthetic_mnist(10000, seed=2024, offset=n)
    Xd = D.upload_rows(tr.compact().X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    out = {}
    for wss in (1, 2):
        v = []
        for rep in range(R + 1):
            a = torch.zeros(n, dtype=torch.float64, device=dev)
            torch.cuda.synchronize()
            t = time.perf_counter()
            r, _ = D.smo(K, yd, a, SVMParams(wss=wss), n=n)
            torch.cuda.synchronize()
            if rep:
                v.append((time.perf_counter() - t) * 1e3)
        out[wss] = (r, min(v), statistics.median(v), set(np.flatnonzero(a.cpu().numpy() > 1e-8).tolist()))
    del K
    torch.cuda.empty_cache()
    acc = {w: SVC(device="cuda:0", wss=("first" if w == 1 else "second")).fit(tr.compact().X, tr.y)
           .score(te.compact().X, te.y) for w in (1, 2)}
    for wss in (1, 2):
        r, best, med, sv = out[wss]
        print(f"n={n} wss={'first ' if wss == 1 else 'second'}: iterations {r.iterations:6d} | smo best {best:7.2f} ms "
              f"median {med:7.2f} ms ({best * 1e3 / r.iterations:.3f} us/iter) | nSV {len(sv)} | b {r.b:.10f} | "
              f"test acc {acc[wss]:.4f}", flush=True)
    print(f"n={n}: SV sets differ by {len(out[1][3] ^ out[2][3])}", flush=True)
