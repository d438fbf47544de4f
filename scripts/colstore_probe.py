"""The narrow column store alone (the decomposition's miss fill): svmd_decomp_gemv_u8 through the column
cache (SVM355_GEMV_VIA_CACHE=1: plan + store of m columns + cached-column sum) on n MNIST-shaped rows,
best of 10 per m, against the same sum by the GEMV.  argv: n [m ...]."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ms = [int(v) for v in sys.argv[2:]] or [1, 8, 32, 64]
tr = synthetic_mnist(n, seed=4).compact()
dev = torch.device("cuda:0")
Xu = D.upload_u8(tr.X, dev)
mmd = torch.empty(2 * tr.d, dtype=torch.float64, device=dev)
D.minmax_u8(Xu, out=mmd)
mm = mmd.cpu().numpy()
mn, mx = mm[: tr.d].copy(), mm[tr.d:].copy()
rng = np.random.default_rng(0)
label = os.environ.get("PROBE_LABEL", "")
for via in ("1", "0"):
    os.environ["SVM355_GEMV_VIA_CACHE"] = via
    for m in ms:
        cols = np.sort(rng.choice(n, size=m, replace=False)).astype(np.int32)
        coef = rng.uniform(-1, 1, size=m)
        best = 1e9
        for _ in range(10):
            torch.cuda.synchronize()
            t = time.perf_counter()
            D.decomp_gemv_u8(Xu, mn, mx, 0.00125, cols, coef)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        print(f"{label} n={n} m={m} {'cache (plan+store+sum)' if via == '1' else 'gemv'}: {best * 1e3:.3f} ms "
              f"({n * 832 / best / 1e12:.2f} TB/s of int8 rows at kq 832)", flush=True)
