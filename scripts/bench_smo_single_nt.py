"""Single-workgroup SMO at cascade-merge sizes with narrow workgroups (SVM355_SMO_SINGLE_NT = 64 / 128:
one or two waves, no or one cheap barrier) against the shipped 512 threads; same Gram, same trajectory
required.  Best of 5."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
os.environ["SVM355_SMO"] = "single"
for n in [int(v) for v in (sys.argv[1:] or ["600", "1000", "1400", "2000"])]:
    tr = synthetic_mnist(n, seed=2024)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    ref = None
    for nt in (64, 128, 256, 512):
        if n > nt * 16:
            continue
        os.environ["SVM355_SMO_SINGLE_NT"] = str(nt)
        best = 1e9
        for _ in range(5):
            a = torch.zeros(n, dtype=torch.float64, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r, _ = D.smo(K, yd, a, SVMParams(), n=n)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e3)
        ref = ref or (r.iterations, r.b)
        flag = "" if (r.iterations, r.b) == ref else " TRAJECTORY DIFFERS"
        print(f"n={n:5d} single NT={nt:4d}: {best:7.2f} ms  iters {r.iterations:5d}  us/iter "
              f"{best * 1e3 / max(1, r.iterations):.3f}{flag}", flush=True)
