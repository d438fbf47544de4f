"""`reps` decomposition fits of synthetic_mnist(n, seed) -- a short program for rocprofv3 (the solver's
knobs come from the environment, e.g. SVM355_DECOMP_SHRINK=0)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 2024
tr = synthetic_mnist(n, seed=seed).compact()
for _ in range(reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    m = SVC(device="cuda:0", solver="decomp", max_iter=10_000_000).fit(tr.X, tr.y)
    torch.cuda.synchronize()
    tm = m.timings_
    print(f"n={n} fit {1e3 * (time.perf_counter() - t):.2f} ms outer {tm.get('outer_iterations')} inner "
          f"{tm.get('inner_iterations')} nsv {len(m.support_)} unshrinks {tm.get('unshrinks')} passes "
          f"{tm.get('shrink_passes')} min_active {tm.get('min_active')} repacks {tm.get('repacks')}", flush=True)
