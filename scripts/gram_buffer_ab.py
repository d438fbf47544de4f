"""Gram time by output buffer: torch-allocated (rbf_gram_sym(out=K)) vs the library-owned Gram of a
full fit (D.train timing gram_ms), alternating in one process, best and median of R."""
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
n = 60000
tr = synthetic_mnist(n, seed=2024)
Xd = D.upload_rows(tr.compact().X, dev)
mn, mx, sqn = D.minmax_scale_(Xd, 784)
yd = torch.from_numpy(tr.y).to(dev)
K = None
t_torch, t_lib, t_lib_smo = [], [], []
for rep in range(6):
    torch.cuda.synchronize()
    t = time.perf_counter()
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, out=K)
    torch.cuda.synchronize()
    t_torch.append((time.perf_counter() - t) * 1e3)
    a = torch.zeros(n, dtype=torch.float64, device=dev)
    r, tm = D.train(Xd, sqn, yd, a, SVMParams(), mn=mn, mx=mx, kcache="full")
    t_lib.append(tm["gram_ms"])
    t_lib_smo.append(tm["smo_ms"])
for name, v in (("torch buffer (rbf_gram_sym)", t_torch), ("train(kcache=full) gram_ms", t_lib),
                ("train smo_ms", t_lib_smo)):
    print(f"{name}: best {min(v[1:]):.2f} median {statistics.median(v[1:]):.2f} ms  all {[round(x, 2) for x in v]}")
