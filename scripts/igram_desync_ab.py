"""Exact-integer Gram at n = 60000 with co-resident workgroups phase-offset (SVM355_IGRAM_DESYNC=mode:us,
read per launch): mode 1 = blockIdx in [256, 512) start late, 2 = odd blockIdx < 512, 3 = odd per-XCD
sequence index < 512.  Alternating rounds, best and median of R per setting; the Gram must be bit-identical."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
tr = synthetic_mnist(n, seed=2024)
Xd = D.upload_rows(tr.compact().X, dev)
mn, mx, sqn = D.minmax_scale_(Xd, 784)
settings = ["", "1:5", "1:10", "2:5", "2:10", "3:5", "3:10", "1:15", "2:15"]
K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, out=None)
ref = K.clone() if n <= 30000 else K[::997].clone()
times = {s: [] for s in settings}
for rnd in range(5):
    for s in settings:
        if s:
            os.environ["SVM355_IGRAM_DESYNC"] = s
        else:
            os.environ.pop("SVM355_IGRAM_DESYNC", None)
        torch.cuda.synchronize()
        t = time.perf_counter()
        K, info = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, out=K)
        torch.cuda.synchronize()
        times[s].append((time.perf_counter() - t) * 1e3)
        got = K if n <= 30000 else K[::997]
        assert torch.equal(got, ref), f"setting {s}: Gram differs"
    print(f"round {rnd} done", flush=True)
for s in settings:
    print(f"n={n} desync {s or 'off':6s}: best {min(times[s]):.2f} ms  median {statistics.median(times[s]):.2f} ms", flush=True)
