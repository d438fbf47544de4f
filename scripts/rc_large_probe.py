"""Large-n row-cache solves in one process with SVM355_RC_VERBOSE=1: the same n repeated, with and
without a host-side pause before it, to separate allocation / clock / cache-size effects."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
os.environ["SVM355_RC_VERBOSE"] = "1"
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
for n, pauses in [(250000, [0, 0]), (500000, [0, 0, 3, 0]), (1000000, [0, 0])]:
    tr = synthetic_mnist(n, seed=2024).compact()
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    yd = torch.from_numpy(tr.y).to(dev)
    for pz in pauses:
        time.sleep(pz)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        t = time.perf_counter()
        r, _ = D.train(Xd, sqn, yd, a, SVMParams(), mn=mn, mx=mx, kcache="rows")
        torch.cuda.synchronize()
        print(f"n={n} pause {pz}s: {(time.perf_counter() - t) * 1e3:.0f} ms, iters {r.iterations}", flush=True)
    del Xd, a, yd, sqn
    torch.cuda.empty_cache()
