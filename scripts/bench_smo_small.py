"""Per-iteration cost of the SMO solvers on small problems (cascade-sized): single workgroup vs the
multi-workgroup persistent kernel at several grid sizes, same Gram, same trajectory required."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
for n in [int(v) for v in (sys.argv[1:] or ["1500", "3500", "6000", "8700", "15000"])]:
    tr = synthetic_mnist(n, seed=2024)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    modes = [("single", nt) for nt in (256, 512, 1024)] if n <= 8192 else []
    modes += [("persistent", g) for g in (8, 32, 64)]
    ref = None
    for mode, g in modes:
        os.environ["SVM355_SMO"] = mode
        os.environ["SVM355_PSMO_WG"] = str(g if mode == "persistent" else 64)
        os.environ["SVM355_SMO_SINGLE_NT"] = str(g if mode == "single" else 256)
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
        print(f"n={n:6d} {mode:>10} G<={g:3d}: {best:8.2f} ms  iters {r.iterations:6d}  us/iter "
              f"{best * 1e3 / max(1, r.iterations):.3f}{flag}", flush=True)

if os.environ.get("PSMO_STAMPS"):
    os.environ["SVM355_PSMO_STAMP"] = "1"
    os.environ["SVM355_SMO"] = "single"
    for n in (1500, 3500):
        tr = synthetic_mnist(n, seed=2024)
        Xd = D.upload_rows(tr.X, dev)
        mn, mx, sqn = D.minmax_scale_(Xd, 784)
        K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
        yd = torch.from_numpy(tr.y).to(dev)
        for nt in (256, 512, 1024):
            os.environ["SVM355_SMO_SINGLE_NT"] = str(nt)
            a = torch.zeros(n, dtype=torch.float64, device=dev)
            D.smo(K, yd, a, SVMParams(), n=n)
            torch.cuda.synchronize()
