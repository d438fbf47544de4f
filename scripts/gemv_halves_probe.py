#!/usr/bin/env python3
"""The f-update GEMV alone at 60k for 1 / 2 / 3 / 5 / 8 column halves (64 / 128 / 192 / 320 / 512 moved
columns), 6 calls each in that order: under rocprofv3 --kernel-trace the GEMV kernel's durations per m
show how its time grows with the halves a workgroup walks."""
import sys

import numpy as np
import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

tr = synthetic_mnist(60000, seed=2024).compact()
dev = torch.device("cuda", 0)
Xu = D.upload_u8(tr.X, dev)
mmd = torch.empty(2 * tr.d, dtype=torch.float64, device=dev)
mn, mx = D.minmax_u8(Xu, out=mmd)
mm = mmd.cpu().numpy()
rng = np.random.default_rng(1)
for m in (64, 128, 160, 192, 320, 512):
    cols = np.sort(rng.choice(60000, size=m, replace=False)).astype(np.int32)
    coef = rng.uniform(-1, 1, size=m)
    for _ in range(6):
        D.decomp_gemv_u8(Xu, mm[: tr.d].copy(), mm[tr.d:].copy(), 0.00125, cols, coef)
    torch.cuda.synchronize()
    print("m", m, flush=True)
