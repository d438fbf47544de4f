"""Idle -> busy ramp: after a 50 ms host sleep, run ~W ms of all-CU work (a torch fp64 GEMM), then the
Gram (HIP events around the Gram only)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
n = 60000
tr = synthetic_mnist(n, seed=2024)
Xd = D.upload_rows(tr.compact().X, dev)
mn, mx, sqn = D.minmax_scale_(Xd, 784)
K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
A = torch.randn(2048, 2048, dtype=torch.float64, device=dev)


def run(busy_reps):
    time.sleep(0.05)
    eb0, eb1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    eb0.record()
    for _ in range(busy_reps):
        A @ A
    eb1.record()
    e0.record()
    D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, out=K)
    e1.record()
    torch.cuda.synchronize()
    return eb0.elapsed_time(eb1), e0.elapsed_time(e1)


for reps in (0, 1, 2, 4, 8, 0):
    v = [run(reps) for _ in range(4)]
    print(f"busy GEMMs {reps}: busy {sorted(b for b, _ in v)[1]:.2f} ms, then gram " +
          " ".join(f"{g:.2f}" for _, g in v), flush=True)
