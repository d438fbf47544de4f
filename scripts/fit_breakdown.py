"""Wall-clock breakdown of one SVC.fit on the GPU (60k synthetic MNIST), phase by phase."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from svm355 import SVC  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
tr = synthetic_mnist(n, seed=2024)
dev = torch.device("cuda:0")
SVC(device="cuda:0").fit(tr.X, tr.y)  # warm-up (allocator, code objects)
for rep in range(2):
    T = {}
    torch.cuda.synchronize()
    t = time.perf_counter()

    def mark(k):
        global t
        torch.cuda.synchronize()
        now = time.perf_counter()
        T[k] = round((now - t) * 1e3, 3)
        t = now

    Xd = D.upload_rows(tr.X, dev); mark("upload")
    yd = torch.from_numpy(np.ascontiguousarray(tr.y, dtype=np.int32)).to(dev); mark("y_h2d")
    mn, mx, sqn = D.minmax_scale_(Xd, 784); mark("minmax_scale")
    alpha = torch.zeros(n, dtype=torch.float64, device=dev); mark("alpha0")
    res, tm = D.train(Xd, sqn, yd, alpha, SVC().params, mn=mn, mx=mx); mark("train")
    a = alpha.cpu().numpy(); mark("alpha_d2h")
    sup = np.flatnonzero(a > 1e-8); mark("sv_extract")
    idx = torch.from_numpy(sup).to(dev); Xs = D.gather_rows(Xd, idx); mark("gather_sv")
    svc = SVC(device="cuda:0")
    t0 = time.perf_counter(); svc.fit(tr.X, tr.y); torch.cuda.synchronize(); full = (time.perf_counter() - t0) * 1e3
    print(f"rep {rep}: {T} native={tm} | SVC.fit total {full:.3f} ms timings_={svc.timings_}", flush=True)
