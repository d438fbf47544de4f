"""The decomposition solver past the former 2,097,152-row cap (streamed selection blocks): MNIST-shaped
synthetic rows at 3M, one cold and two warm fits; the solve's shape and time."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from svm355 import SVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3_000_000
max_iter = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000  # past the reference's 100,000 at this size
t = time.perf_counter()
tr = synthetic_mnist(n, seed=0).compact()
print(f"data n={n} generated in {time.perf_counter() - t:.1f} s", flush=True)
for k in range(2):
    torch.cuda.synchronize()
    t = time.perf_counter()
    m = SVC(device="cuda:0", solver="decomp", max_iter=max_iter).fit(tr.X, tr.y)
    torch.cuda.synchronize()
    tm = m.timings_
    print(f"fit {k}: {time.perf_counter() - t:.3f} s (solve {tm['smo_ms'] / 1e3:.3f} s) outer {tm['outer_iterations']} "
          f"pair updates {tm['inner_iterations']} capacity {tm['working_set']} SVs {m.support_.size} "
          f"b {m.b_:.10f} {m.stop_reason_} kcache {tm['kcache']}", flush=True)
