"""A/B of the row-cache solver's K12 source (SVM355_RC_K12 = compute | cache): K(i_high, i_low)
recomputed from the int8 rows every iteration, or read from a cached row filled two or more epochs
earlier (smo.hip CachedRows K12C).  Same process, alternating, best of REPS per variant; the
trajectories must be identical (iterations, b, alphas)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

sizes = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "60000,120000,250000").split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
for n in sizes:
    X = synthetic_mnist(n, seed=2024).compact()
    best, ref = {}, None
    for rep in range(reps + 1):  # the first round warms the slab / context
        for mode in ("compute", "cache"):
            os.environ["SVM355_RC_K12"] = mode
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m = SVC(device="cuda:0", kcache="rows").fit(X.X, X.y)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            key = (m.n_iter_, m.b_, m.alpha_.tobytes())
            if ref is None:
                ref = key
            assert key == ref, f"n={n} {mode}: trajectory differs (iterations {m.n_iter_} vs {ref[0]}, b {m.b_} vs {ref[1]})"
            if rep:
                best[mode] = min(best.get(mode, 1e30), dt)
    print(f"n={n}: iterations {ref[0]} b {ref[1]:.12f} | K12 computed {best['compute']:.1f} ms | "
          f"K12 from cached rows {best['cache']:.1f} ms | {best['compute'] / best['cache']:.3f}x", flush=True)
os.environ.pop("SVM355_RC_K12", None)
