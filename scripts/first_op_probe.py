"""Which first GPU operation of a fresh process pays the one-off ~100 ms (cold first fit): each step
timed alone (synchronised), in the order given on the command line.
  steps: h2d (tiny host-to-device copy), ctx (svm355 device context), native (one svm355 kernel),
         torch (one PyTorch kernel), fit (SVC.fit at 60k)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from svm355 import SVC  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

order = sys.argv[1].split(",") if len(sys.argv) > 1 else ["h2d", "ctx", "native", "torch", "fit"]
dev = torch.device("cuda:0")
tr = synthetic_mnist(60000, seed=2024).compact() if "fit" in order else None
t0 = time.perf_counter()
torch.cuda.init()
print(f"torch.cuda.init {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
small = np.arange(64 * 16, dtype=np.uint8).reshape(64, 16)
x = None
for step in order:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if step == "h2d":
        x = torch.from_numpy(small).to(dev)
    elif step == "ctx":
        D._ctx_for(x if x is not None else torch.empty(1, device=dev))
    elif step == "native":
        xs = x if x is not None else torch.from_numpy(small).to(dev)
        D.minmax_u8(xs)
    elif step == "torch":
        torch.ones(16, device=dev).add_(1.0)
    elif step == "fit":
        SVC(device="cuda:0").fit(tr.X, tr.y)
    torch.cuda.synchronize()
    print(f"{step:7s} {1e3 * (time.perf_counter() - t0):8.1f} ms", flush=True)
