"""A/B of the persistent SMO's record polling (SVM355_PSMO_POLL2 = 1: two polls in flight, 0: one),
interleaved rounds on one resident Gram per size; identical trajectories required.

    python scripts/psmo_poll.py [n ...]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
for n in [int(v) for v in sys.argv[1:]] or [60000, 8700, 3500]:
    tr = synthetic_mnist(n, seed=2024)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    os.environ["SVM355_SMO"] = "persistent"
    modes = ["0", "1", "-4", "-8", "-16"]
    res = {m: [] for m in modes}
    sig = {}
    for rnd in range(4):
        for p2 in modes:
            os.environ["SVM355_PSMO_POLL2"] = p2
            a = torch.zeros(n, dtype=torch.float64, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r, _ = D.smo(K, yd, a, SVMParams(), n=n)
            torch.cuda.synchronize()
            res[p2].append((time.perf_counter() - t0) * 1e3)
            sig[p2] = (r.iterations, r.b)
    it = sig["0"][0]
    for p2, v in res.items():
        print(f"n={n:6d} poll2={p2}: best {min(v):7.2f} ms  {min(v) * 1e3 / it:.3f} us/iter  iterations {it}  "
              f"same trajectory: {sig[p2] == sig['0']}", flush=True)
    del K
