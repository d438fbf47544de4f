"""A/B of the persistent SMO at the headline shape: best-of-R solve time on one resident 60k Gram.
Run once per built variant of smo.hip (record store scope)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = 60000
dev = torch.device("cuda:0")
tr = synthetic_mnist(n, seed=2024).compact()
Xd = D.upload_rows(tr.X, dev)
mn, mx, sqn = D.minmax_scale_(Xd, 784)
K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
yd = torch.from_numpy(tr.y).to(dev)
best = 1e9
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 7):
    a = torch.zeros(n, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    r, _ = D.smo(K, yd, a, SVMParams(), n=n)
    torch.cuda.synchronize()
    best = min(best, time.perf_counter() - t)
print(f"n={n} iters {r.iterations} b {r.b!r} best smo {best * 1e3:.2f} ms = {best * 1e6 / r.iterations:.3f} us/iter", flush=True)
