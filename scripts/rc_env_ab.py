"""A/B of a row-cache solver switch read from the environment at each solve, e.g.
    python scripts/rc_env_ab.py SVM355_RC_LAYOUT rows,sliced 60000,250000 2
Same process, the variants alternate, best of REPS per variant after one warm-up round; every
fit must follow the same trajectory (iterations, b, alphas)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

var, vals = sys.argv[1], sys.argv[2].split(",")
sizes = [int(v) for v in sys.argv[3].split(",")]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
for n in sizes:
    X = synthetic_mnist(n, seed=2024).compact()
    best, ref = {}, None
    for rep in range(reps + 1):
        for v in vals:
            os.environ[var] = v
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m = SVC(device="cuda:0", kcache="rows").fit(X.X, X.y)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            key = (m.n_iter_, m.b_, m.alpha_.tobytes())
            if ref is None:
                ref = key
            assert key == ref, f"n={n} {var}={v}: trajectory differs ({m.n_iter_} vs {ref[0]} iterations)"
            if rep:
                best[v] = min(best.get(v, 1e30), dt)
    print(f"n={n}: iterations {ref[0]} b {ref[1]:.12f} | " + " | ".join(f"{var}={v} {best[v]:.1f} ms" for v in vals),
          flush=True)
os.environ.pop(var, None)
