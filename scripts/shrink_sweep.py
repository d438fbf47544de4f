#!/usr/bin/env python3
"""Decomposition fit time with and without shrinking (decomp_shrink.h), in one process.
Usage: shrink_sweep.py N[,N..] 'K=V K=V' 'K=V' ...  ('' = the defaults; SVM355_DECOMP_SHRINK=0 = off).
Prints the median of the warm fits, the shrink counters, and whether the SV set equals the first
setting's (the trajectories differ by design; the stop test is the same)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from svm355 import SVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

sizes = [int(s) for s in sys.argv[1].split(",")]
settings = sys.argv[2:] or [""]
seed = int(os.environ.get("SWEEP_SEED", "2024"))
max_iter = int(os.environ.get("SWEEP_MAX_ITER", "100000"))
dev = torch.device("cuda", 0)
for n in sizes:
    tr = synthetic_mnist(n, seed=seed).compact()
    reps = 7 if n <= 100000 else 3
    ref = None
    for st in settings:
        kv = dict(x.split("=", 1) for x in st.split())
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            m = SVC(device="cuda:0", solver="decomp", max_iter=max_iter).fit(tr.X, tr.y)
            torch.cuda.synchronize(dev)
            ts.append(1e3 * (time.perf_counter() - t))
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        sv = tuple(m.support_.tolist())
        ref = ref or sv
        tm = m.timings_
        print(f"n={n} [{st or 'defaults'}]: median {np.median(ts[1:]):.2f} ms min {min(ts[1:]):.2f} smo "
              f"{tm.get('smo_ms', 0):.2f} outer {tm.get('outer_iterations')} inner {tm.get('inner_iterations')} "
              f"nsv {len(sv)} b {m.b_:.10f} stop {getattr(m, 'stop_reason_', '?')} "
              f"unshrinks {tm.get('unshrinks')} passes {tm.get('shrink_passes')} min_active {tm.get('min_active')} "
              f"repacks {tm.get('repacks')} newton {tm.get('newton_steps')} same_svs={sv == ref}", flush=True)
