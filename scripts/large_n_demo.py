"""Beyond the resident-Gram limit: train on n synthetic MNIST rows whose n x n FP64 Gram does not fit
in one MI355X's HBM (n = 250k -> 500 GB), via the on-demand HBM row cache (rowcache.hip)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVC  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 250000
t0 = time.perf_counter()
tr = synthetic_mnist(n, seed=2024)
te = synthetic_mnist(10000, seed=2024, offset=n)
print(f"data: {n} x 784 generated in {time.perf_counter() - t0:.1f} s; full Gram would need "
      f"{n * n * 8 / 1e9:.0f} GB, fits: {D.gram_fits(n, 'cuda:0')}", flush=True)
Xu8 = tr.compact().X  # uint8 pixels, widened on the device
wss_list = (sys.argv[2] if len(sys.argv) > 2 else "first").split(",")  # e.g. "first,second"
for wss, rep in [(w, r) for w in wss_list for r in range(2)]:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = SVC(device="cuda:0", wss=wss).fit(Xu8, tr.y)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"[{wss}] fit {dt * 1e3:.1f} ms: kcache={m.timings_['kcache']} gram={m.timings_['gram_path']} "
          f"iterations={m.n_iter_} n_sv={len(m.support_)} b={m.b_:.12f} stop={m.stop_reason_} timings={m.timings_}",
          flush=True)
print(f"test accuracy {m.score(te.X, te.y):.4f}", flush=True)
