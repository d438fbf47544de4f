#!/usr/bin/env python3
"""L2 prefetch of K(W, W) for the inner solve: 60k / 250k decomposition fits with
SVM355_DECOMP_PF_H helper workgroups on the inner solve's XCD reading the first SVM355_DECOMP_PF_ROWS rows
of K(W, W) before / while the solve runs.  The knobs exist only in commit 2254cc6 (measured, not kept:
profiles/r5_inner_chain_variants.txt).  Prints the median fit time per setting and checks the model
(SV count, b, iterations) is the same as without helpers (they only read)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from svm355 import SVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

sizes = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "60000").split(",")]
settings = [(0, 1024), (4, 1024), (16, 1024), (31, 1024), (16, 512), (31, 512), (31, 384)]
dev = torch.device("cuda", 0)
for n in sizes:
    tr = synthetic_mnist(n, seed=2024).compact()
    ref = None
    reps = 7 if n <= 60000 else 3
    for h, rows in settings:
        os.environ["SVM355_DECOMP_PF_H"] = str(h)
        os.environ["SVM355_DECOMP_PF_ROWS"] = str(rows)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            m = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
            torch.cuda.synchronize(dev)
            ts.append(1e3 * (time.perf_counter() - t))
        sig = (len(m.support_), float(m.b_), int(m.n_iter_), m.alpha_.tobytes().__hash__())
        if ref is None:
            ref = sig
        print(f"n={n} PF_H={h:2d} PF_ROWS={rows:4d}: median {np.median(ts[1:]):.2f} ms  min {min(ts[1:]):.2f}  "
              f"smo {m.timings_.get('smo_ms', 0):.2f}  same_model={sig == ref}", flush=True)
