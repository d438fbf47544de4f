#!/usr/bin/env python3
"""How often the decomposition's f update recomputes a kernel column it has computed before (design input
of the column cache): per outer iteration the moved columns (trace), then the uses,
the distinct columns, and the share of uses that a cache of C columns would serve.

    python scripts/decomp_column_reuse.py 60000 250000 1000000
"""
import sys

import numpy as np
import torch

from svm355 import SVMParams
from svm355 import _native as N
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
    alpha = torch.empty(n, dtype=torch.float64, device=dev)
    t = N.DecompTrace(2000, 0)
    res, tm = D.train_decomp(Xu, yd, alpha, SVMParams(), mm[: tr.d], mm[tr.d:], trace=t)
    recs = t.records()
    uses = sum(r["moved"] for r in recs)
    seen, hits = set(), 0
    first = []
    for r in recs:
        c = r["cols"].tolist()
        hits += sum(1 for x in c if x in seen)
        seen.update(c)
        first.append(len(seen))
    print(f"n={n}: outer {len(recs)} pair updates {tm['inner_iterations']} column uses {uses} distinct {len(seen)} "
          f"reuse share {hits / max(uses, 1):.3f} (unbounded cache); stop {res.stop_reason}", flush=True)
    del Xu, yd, alpha
    torch.cuda.empty_cache()
