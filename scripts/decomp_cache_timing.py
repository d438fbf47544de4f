#!/usr/bin/env python3
"""Decomposition fit time with the column cache off / on (SVM355_DECOMP_CCACHE, read per fit) at the
sizes of argv: best of 3 fits after a warm-up, the alpha of both compared bit for bit
(SVM355_DECOMP_CCACHE_FIXED=0|1: that setting only, for a profile; SVM355_TIMING_VAR: the variable
toggled instead of SVM355_DECOMP_CCACHE, e.g. SVM355_DECOMP_WCOLS; SVM355_TIMING_VALUES: its values,
comma-separated, instead of 0 and 1).

    python scripts/decomp_cache_timing.py 60000 250000 1000000
"""
import os
import sys
import time

import numpy as np
import torch

from svm355 import SVMParams
from svm355.ops import device as D
from svm355.utils.data import synthetic_mnist

dev = torch.device("cuda:0")
for n in [int(a) for a in sys.argv[1:]]:
    tr = synthetic_mnist(n, seed=2024).compact()
    Xu = D.upload_u8(tr.X, dev)
    mmd = torch.empty(2 * tr.d, dtype=torch.float64, device=dev)
    D.minmax_u8(Xu, out=mmd)
    mm = mmd.cpu().numpy()
    yd = torch.from_numpy(tr.y).to(dev)
    res = {}
    flags = (os.environ["SVM355_DECOMP_CCACHE_FIXED"],) if "SVM355_DECOMP_CCACHE_FIXED" in os.environ else ("0", "1")
    if "SVM355_TIMING_VALUES" in os.environ:
        flags = tuple(os.environ["SVM355_TIMING_VALUES"].split(","))
    for flag in flags:
        os.environ[os.environ.get("SVM355_TIMING_VAR", "SVM355_DECOMP_CCACHE")] = flag
        best = 1e30
        for rep in range(4):
            alpha = torch.empty(n, dtype=torch.float64, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r, tm = D.train_decomp(Xu, yd, alpha, SVMParams(), mm[: tr.d], mm[tr.d:])
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if rep:
                best = min(best, dt)
        res[flag] = (alpha.cpu().numpy(), r.b, r.iterations, tm["outer_iterations"], best)
        print(f"n={n} cache={flag}: fit {best * 1e3:.1f} ms outer {tm['outer_iterations']} pair updates "
              f"{r.iterations} b {r.b:.12f} stop {r.stop_reason}", flush=True)
    if set(res) != {"0", "1"}:
        continue
    same = np.array_equal(res["0"][0], res["1"][0]) and res["0"][1:4] == res["1"][1:4]
    print(f"n={n}: speedup {res['0'][4] / res['1'][4]:.2f}x, alpha bit-identical {same}", flush=True)
    del Xu, yd
    torch.cuda.empty_cache()
