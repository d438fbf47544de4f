"""Cost of a warm start on a resident Gram at cascade sizes: a re-solve from the optimal alphas
stops at its first selection, so its time is the warm-f setup plus fixed overhead.  Best of R.
Run with SVM355_LIB_DIR pointing at another build for an A/B."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
tag = os.environ.get("TAG", "")
for n in (3000, 9000, 30000):
    tr = synthetic_mnist(n, seed=2024)
    Xd = D.upload_rows(tr.compact().X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    a = torch.zeros(n, dtype=torch.float64, device=dev)
    r0, _ = D.smo(K, yd, a, SVMParams(), n=n)
    nz = int((a != 0).sum())
    best = 1e9
    for _ in range(10):
        w = a.clone()
        torch.cuda.synchronize()
        t = time.perf_counter()
        r, _ = D.smo(K, yd, w, SVMParams(), n=n, warm=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    print(f"{tag} n={n} nnz={nz}: warm re-solve {best * 1e3:.3f} ms, iterations {r.iterations}, b {r.b!r} (cold b {r0.b!r})",
          flush=True)
