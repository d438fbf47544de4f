#!/usr/bin/env python3
"""Column-store timing: the f update of m columns through the column cache (every column a miss) on n
synthetic MNIST rows, repeated; run under rocprofv3 --kernel-trace --stats for the per-kernel times.

    SVM355_GEMV_VIA_CACHE=1 python scripts/colstore_bench.py 1000000 1 8 32 64
"""
import sys

import numpy as np
import torch

from svm355.ops import device as D
from svm355.utils.data import synthetic_mnist

n = int(sys.argv[1])
dev = torch.device("cuda:0")
tr = synthetic_mnist(n, seed=7).compact()
Xu = D.upload_u8(tr.X, dev)
mmd = torch.empty(2 * tr.d, dtype=torch.float64, device=dev)
D.minmax_u8(Xu, out=mmd)
mm = mmd.cpu().numpy()
rng = np.random.default_rng(1)
for m in [int(a) for a in sys.argv[2:]]:
    cols = np.sort(rng.choice(n, size=m, replace=False)).astype(np.int32)
    coef = rng.uniform(-1, 1, size=m)
    for _ in range(5):
        out = D.decomp_gemv_u8(Xu, mm[: tr.d], mm[tr.d:], 0.00125, cols, coef, 0, n)
    print(f"m={m}: f[0..3] {out[:3]}", flush=True)
