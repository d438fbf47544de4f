"""One-vs-rest over all 10 digits on one resident Gram: class solves one after another, concurrently
on separate streams (OneVsRestSVC(solver="streams", concurrent_solves=...)), and batched in one
launch with a team per XCD (solver="batched"); identical models required.

    python scripts/bench_ovr.py [n]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import OneVsRestSVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
tr = synthetic_mnist(n, seed=2024).compact()
te = synthetic_mnist(10000, seed=2024, offset=n).compact()
ref = None
for rnd in range(2):
    for cs in (1, 4, 8, "batched"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kw = {"solver": "batched"} if cs == "batched" else {"solver": "streams", "concurrent_solves": cs}
        m = OneVsRestSVC(device="cuda:0", **kw).fit(tr.X, tr.labels)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        sig = (tuple(m.n_iter_.tolist()), tuple(m.intercepts_b_.tolist()))
        ref = ref or sig
        if rnd == 1:
            print(f"n={n} {'batched (XCD teams)' if cs == 'batched' else f'streams x{cs}':20s}: fit {dt:8.1f} ms  (gram {m.timings_['gram_ms']:.1f}, "
                  f"smo all classes {m.timings_['smo_ms_all_classes']:.1f})  iterations {sum(m.n_iter_)}  "
                  f"identical={sig == ref}  accuracy={m.score(te.X, te.labels):.4f}", flush=True)
