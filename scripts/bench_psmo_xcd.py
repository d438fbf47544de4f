"""Device-wide vs XCD-local persistent SMO (and the single-workgroup solver) across n; same Gram,
same trajectory required.  Best of 3 runs."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
for n in [int(v) for v in (sys.argv[1:] or ["3500", "8700", "15000", "30000", "60000"])]:
    tr = synthetic_mnist(n, seed=2024)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    modes = [("persistent", "0", "512"), ("persistent", "1", "512"), ("persistent", "1", "256")]
    if n <= 8192:
        modes.append(("single", "0", "512"))
    ref = None
    for mode, xcd, nt in modes:
        os.environ.update({"SVM355_SMO": mode, "SVM355_PSMO_XCD": xcd, "SVM355_PSMO_NT": nt})
        best = 1e9
        for _ in range(3):
            a = torch.zeros(n, dtype=torch.float64, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r, _ = D.smo(K, yd, a, SVMParams(), n=n)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e3)
        ref = ref or (r.iterations, r.b)
        flag = "" if (r.iterations, r.b) == ref else " TRAJECTORY DIFFERS"
        print(f"n={n:6d} {mode:>10} xcd={xcd} NT={nt}: {best:8.2f} ms  iters {r.iterations:6d}  "
              f"us/iter {best * 1e3 / max(1, r.iterations):.3f}{flag}", flush=True)
    del K
    torch.cuda.empty_cache()
