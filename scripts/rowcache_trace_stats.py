"""How many kernel rows does an SMO touch?  Runs the row-cache solver on n synthetic MNIST rows with
the (i_high, i_low) trace and counts distinct rows and 2-way-LRU misses for a few cache sizes."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402


def lru_misses(trace, slots, window=None):
    """2-way LRU misses of the pair sequence (the device directory's policy); with window=(a, b)
    only iterations a <= k < b are counted."""
    nsets = slots // 2
    tags = -np.ones((nsets, 2), np.int64)
    mru = np.zeros(nsets, np.int8)
    miss = 0
    for k, (ih, il) in enumerate(trace):
        count = window is None or window[0] <= k < window[1]
        keep = -1
        for r in (ih, il):
            s = r % nsets
            if tags[s, 0] == r:
                mru[s] = 0
                continue
            if tags[s, 1] == r:
                mru[s] = 1
                continue
            v = 1 - mru[s]
            if keep == (s, v):
                v = 1 - v
            tags[s, v] = r
            mru[s] = v
            keep = (s, v)
            miss += count
    return miss


dev = torch.device("cuda:0")
for n in [int(x) for x in (sys.argv[1:] or ["60000", "120000", "250000"])]:
    tr = synthetic_mnist(n, seed=2024).compact()
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    yd = torch.from_numpy(tr.y).to(dev)
    a = torch.zeros(n, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    r, tm = D.train(Xd, sqn, yd, a, SVMParams(), mn=mn, mx=mx, kcache="rows", trace_cap=200000)
    ms = (time.perf_counter() - t) * 1e3
    trc = tm["trace"]
    distinct = len(np.unique(trc))
    line = f"n={n}: iters {r.iterations} b {r.b:.12f} nsv {int((a > 1e-8).sum())} time {ms:.0f} ms " \
           f"({ms * 1e3 / r.iterations:.1f} us/iter) distinct rows {distinct}"
    for slots in (4096, 16384):
        line += f" | misses@{slots} {lru_misses(trc, slots)}"
    # the phase stamps (SVM355_PSMO_STAMP=1) sample 2000 epochs from SVM355_PSMO_STAMP_FROM (200)
    w0 = int(os.environ.get("SVM355_PSMO_STAMP_FROM", "200")) - 1
    line += f" | misses@16384 in stamp window {lru_misses(trc, 16384, (w0, w0 + 2000))}"
    print(line, flush=True)
