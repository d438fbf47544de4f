#!/usr/bin/env python3
"""Where a fresh process's device initialisation goes: the first PyTorch GPU
operation and svmd_create (DeviceContext.get: streams, the 32 MB copy-engine warm copy, one warm-up
launch per translation unit) timed apart, then one 60k fit.  Run twice in a row on a fresh box -- the
first process on the box pays what the second does not -- and under rocprofv3 --runtime-trace to split
svmd_create per HIP call (scripts/rocpd_api.py)."""
import sys
import time

t0 = time.perf_counter()
import torch  # noqa: E402

t1 = time.perf_counter()
sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from svm355 import SVC  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda", 0)
t2 = time.perf_counter()
torch.zeros(1, dtype=torch.uint8).to(dev)
torch.cuda.synchronize(dev)
t3 = time.perf_counter()
D.DeviceContext.get(dev)
torch.cuda.synchronize(dev)
t4 = time.perf_counter()
tr = synthetic_mnist(60000, seed=2024).compact()
t5 = time.perf_counter()
SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
torch.cuda.synchronize(dev)
t6 = time.perf_counter()
print(f"import torch {1e3 * (t1 - t0):.1f} ms | first torch GPU op {1e3 * (t3 - t2):.1f} ms | "
      f"svmd_create {1e3 * (t4 - t3):.1f} ms | first 60k fit {1e3 * (t6 - t5):.1f} ms", flush=True)
