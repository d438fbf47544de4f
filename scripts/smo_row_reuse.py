"""Kernel-row reuse of the SMO trajectory: for an LRU of R rows, how often are the rows of BOTH
working-set indices (i_high, i_low) already resident?  Decides whether an on-chip (LDS/register)
row cache can take the row loads off the per-iteration critical path.

    python scripts/smo_row_reuse.py [n ...]
"""
import os
import sys
from collections import OrderedDict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402


def lru_stats(trace: np.ndarray, R: int):
    lru: OrderedDict = OrderedDict()
    both = one = 0
    for ih, il in trace.tolist():
        h1, h2 = ih in lru, il in lru
        both += h1 and h2
        one += h1 != h2
        for i in (ih, il):
            lru[i] = True
            lru.move_to_end(i)
        while len(lru) > R:
            lru.popitem(last=False)
    n = max(1, len(trace))
    return both / n, one / n


dev = torch.device("cuda:0")
for n in [int(v) for v in sys.argv[1:]] or [60000, 8700, 3500]:
    tr = synthetic_mnist(n, seed=2024)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    a = torch.zeros(n, dtype=torch.float64, device=dev)
    r, t = D.smo(K, torch.from_numpy(tr.y).to(dev), a, SVMParams(), n=n, trace_cap=200000)
    distinct = len(np.unique(t))
    print(f"n={n}: iterations {r.iterations}, distinct rows {distinct}", flush=True)
    for R in (2, 4, 8, 16, 32, 64, 128):
        b, o = lru_stats(t, R)
        print(f"   LRU {R:4d} rows: both resident {b:6.1%}  one {o:6.1%}  neither {1 - b - o:6.1%}", flush=True)
    del K
