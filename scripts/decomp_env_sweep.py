#!/usr/bin/env python3
"""Decomposition fit time under a list of environment settings, in one process (every run_decomp reads
its knobs per fit).  Usage: decomp_env_sweep.py N[,N..] 'K=V K=V' 'K=V' ...  ('' = the defaults).
Prints the median of the warm fits and whether the model (SV set, b, iterations, alpha bytes) equals the
first setting's."""
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
dev = torch.device("cuda", 0)
for n in sizes:
    tr = synthetic_mnist(n, seed=2024).compact()
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
            m = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
            torch.cuda.synchronize(dev)
            ts.append(1e3 * (time.perf_counter() - t))
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        sig = (len(m.support_), float(m.b_), int(m.n_iter_), hash(m.alpha_.tobytes()))
        ref = ref or sig
        tm = m.timings_
        print(f"n={n} [{st or 'defaults'}]: median {np.median(ts[1:]):.2f} ms min {min(ts[1:]):.2f} smo "
              f"{tm.get('smo_ms', 0):.2f} outer {tm.get('outer_iterations')} inner {tm.get('inner_iterations')} "
              f"nsv {sig[0]} same_model={sig == ref}", flush=True)
