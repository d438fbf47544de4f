"""Wall-clock split of one warm 60k SVC.fit outside the solver (host side of the headline step):
the row upload, y upload, min/max + its read-back, and every step after the solve returns."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from svm355 import SVC
from svm355.ops import device as D
from svm355.utils.data import synthetic_mnist

dev = torch.device("cuda:0")
tr = synthetic_mnist(60000, seed=0).compact()
X, y = tr.X, tr.y
m = SVC(device="cuda:0")
for _ in range(3):
    m.fit(X, y)
torch.cuda.synchronize()


def t(fn, reps=20):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        a = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - a)
    return best * 1e3, r


ms, Xu = t(lambda: D.upload_u8(X, dev))
print(f"upload_u8 47 MB       {ms:.3f} ms ({X.nbytes / ms / 1e6:.1f} GB/s)")
ms, yd = t(lambda: torch.from_numpy(y).to(dev))
print(f"y to device           {ms:.3f} ms")
mmd = torch.empty(2 * X.shape[1], dtype=torch.float64, device=dev)
ms, _ = t(lambda: D.minmax_u8(Xu, out=mmd))
print(f"minmax_u8             {ms:.3f} ms")
ms, _ = t(lambda: mmd.cpu().numpy())
print(f"min/max read-back     {ms:.3f} ms")
alpha = torch.empty(60000, dtype=torch.float64, device=dev)
ms, _ = t(lambda: alpha.cpu().numpy())
print(f"alpha read-back       {ms:.3f} ms")
a = m.alpha_
ms, _ = t(lambda: m._finish(a, y, type("R", (), {"b": m.b_, "iterations": m.n_iter_, "stop_reason": "converged"})()))
print(f"_finish               {ms:.3f} ms")
ms, idx = t(lambda: torch.from_numpy(m.support_).to(dev))
print(f"support ids to device {ms:.3f} ms")
mn, mx = mmd[:784], mmd[784:]
ms, _ = t(lambda: D.sv_rows_u8(Xu, idx, mn, mx))
print(f"sv_rows_u8            {ms:.3f} ms")
ms, _ = t(lambda: torch.from_numpy(m.dual_coef_).to(dev))
print(f"coef to device        {ms:.3f} ms")
for _ in range(3):
    a0 = time.perf_counter(); m.fit(X, y); torch.cuda.synchronize(); w = (time.perf_counter() - a0) * 1e3
    tm = m.timings_
    print(f"fit {w:.3f} ms: upload_preprocess {tm['upload_preprocess_ms']:.3f}, total {tm['total_ms']:.3f}, "
          f"rest {w - tm['upload_preprocess_ms'] - tm['total_ms']:.3f}")
