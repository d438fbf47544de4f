"""The first GPU operation after the 2nd and 3rd cascade fits of a process stalls 15-28 ms (not after
the 1st or the 4th+).  Per fit: the device's free memory (does the process still allocate or free?),
the time of a tiny torch op right after the fit, and the fit's wall time."""
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.parallel.cascade import CascadeSVM  # noqa: E402
from svm355.parallel.rccl import DeviceGroup  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
tr = synthetic_mnist(60000, seed=2024).compact()
g = DeviceGroup(1, "rccl")
x = torch.zeros(1, device=dev)
for fit in range(7):
    free0 = torch.cuda.mem_get_info(0)[0]
    t0 = time.perf_counter()
    CascadeSVM(SVMParams()).fit(tr.X, tr.y, world=1, device="cuda", group=g)
    t1 = time.perf_counter()
    free1 = torch.cuda.mem_get_info(0)[0]
    x.add_(1)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    time.sleep(0.05 if fit == 4 else 0.0)
    print(f"fit {fit}: wall {1e3*(t1-t0):7.2f} ms | free before {free0/2**30:8.2f} GiB after {free1/2**30:8.2f} GiB | "
          f"next torch op {1e3*(t2-t1):7.3f} ms", flush=True)
