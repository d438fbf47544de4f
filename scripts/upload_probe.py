#!/usr/bin/env python3
"""Where the cold fit's extra upload time goes: the steps of SVC._fit_cuda_u8's upload, each synchronised
and timed, in a fresh process after the bench's device initialisation; then the same steps again."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

tr = synthetic_mnist(60000, seed=2024).compact()
dev = torch.device("cuda", 0)
torch.zeros(1, dtype=torch.uint8).to(dev)
D.DeviceContext.get(dev)
torch.cuda.synchronize(dev)
import os  # noqa: E402
pre = os.environ.get("PRE", "")
if pre:  # a large copy before the timed reps: "pageable" / "pinned" source into a scratch device buffer
    t = time.perf_counter()
    scratch = torch.empty(32 << 20, dtype=torch.uint8, device=dev)
    src = torch.empty(32 << 20, dtype=torch.uint8, pin_memory=(pre == "pinned"))
    src.fill_(1)
    scratch.copy_(src, non_blocking=False)
    torch.cuda.synchronize(dev)
    print(f"pre-copy ({pre}) {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
    del scratch
for rep in range(3):
    t = {}

    def mark(k, t0):
        torch.cuda.synchronize(dev)
        t[k] = round((time.perf_counter() - t0) * 1e3, 3)
        return time.perf_counter()

    t0 = time.perf_counter()
    X = np.ascontiguousarray(tr.X, dtype=np.uint8)
    t0 = mark("contig", t0)
    out = D.device_empty(X.shape, torch.uint8, dev)
    t0 = mark("empty", t0)
    ctx = D.DeviceContext.get(out.device)
    h = ctx.bind()
    t0 = mark("bind", t0)
    D.N.check(ctx.lib.svmd_memcpy_h2d(h, D.N.ptr(out), D.N.ptr(X), X.nbytes), "h2d")
    t0 = mark("h2d", t0)
    yd = torch.from_numpy(tr.y).to(dev)
    t0 = mark("y", t0)
    mmd = torch.empty(2 * X.shape[1], dtype=torch.float64, device=dev)
    mn, mx = D.minmax_u8(out, out=mmd)
    t0 = mark("minmax", t0)
    mm = mmd.cpu().numpy()
    t0 = mark("readback", t0)
    print(rep, t, flush=True)
    del out, yd, mmd
