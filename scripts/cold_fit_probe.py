"""Where a COLD first fit's time goes (fresh process): the phases of SVC.fit's first call against the
steady state, plus the cost of the first 28.8 GB allocation and of its first touch measured alone."""
import sys
import time

t_start = time.perf_counter()
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, ".")
from svm355 import SVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
mode = sys.argv[2] if len(sys.argv) > 2 else "fit"
tr = synthetic_mnist(n, seed=2024).compact()
t_import = time.perf_counter()
torch.cuda.init()
torch.cuda.synchronize()
t_init = time.perf_counter()
print(f"imports {1e3 * (t_import - t_start):.1f} ms (incl. data), torch.cuda.init {1e3 * (t_init - t_import):.1f} ms",
      flush=True)
if mode == "alloc":
    ldk = (n + 1) // 2 * 2
    t0 = time.perf_counter()
    buf = torch.empty(n * ldk, dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    buf.fill_(0.0)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    buf.fill_(1.0)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(f"alloc {n}x{ldk} f64 ({n * ldk * 8 / 1e9:.1f} GB): torch.empty {1e3 * (t1 - t0):.1f} ms, first fill "
          f"{1e3 * (t2 - t1):.1f} ms, second fill {1e3 * (t3 - t2):.1f} ms", flush=True)
    del buf
for k in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = SVC(device="cuda:0").fit(tr.X, tr.y)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    tm = {k_: round(v, 2) if isinstance(v, float) else v for k_, v in m.timings_.items()}
    print(f"fit {k}: {1e3 * (t1 - t0):.1f} ms  {tm}  it={m.n_iter_}", flush=True)
