#!/usr/bin/env python3
"""Cold vs warm decomposition fit in a fresh process: the bench's device
initialisation first (an upload + the library context, outside any fit, as bench.py does), then the
first fit and two more, each with its phase split.  Run under rocprofv3 --runtime-trace --kernel-trace
to see which HIP calls and first launches the cold fit pays."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from svm355 import SVC  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
tr = synthetic_mnist(n, seed=2024).compact()
dev = torch.device("cuda", 0)
t = time.perf_counter()
torch.zeros(1, dtype=torch.uint8).to(dev)
D.DeviceContext.get(dev)
torch.cuda.synchronize(dev)
print(f"device init {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
for k in range(3):
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    m = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    torch.cuda.synchronize(dev)
    ms = 1e3 * (time.perf_counter() - t)
    tm = {k2: (round(v, 3) if isinstance(v, float) else v) for k2, v in m.timings_.items()}
    print(f"fit {k}: {ms:.2f} ms  {tm}  marker_t={time.perf_counter_ns()}", flush=True)
