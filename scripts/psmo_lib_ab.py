"""Persistent SMO solve time on resident Grams for ONE library build (SVM355_LIB_DIR selects it):
best / median of R; run alternately per build for an A/B."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
R = int(os.environ.get("REPS", "7"))
tag = os.environ.get("TAG", "")
for n in [int(x) for x in (sys.argv[1:] or ["60000"])]:
    tr = synthetic_mnist(n, seed=2024)
    Xd = D.upload_rows(tr.compact().X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    v = []
    for rep in range(R + 1):
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        t = time.perf_counter()
        r, _ = D.smo(K, yd, a, SVMParams(), n=n)
        torch.cuda.synchronize()
        if rep:
            v.append((time.perf_counter() - t) * 1e3)
    print(f"{tag} n={n}: best {min(v):.2f} median {statistics.median(v):.2f} ms ({min(v) * 1e3 / r.iterations:.3f} "
          f"us/iter), iterations {r.iterations}", flush=True)
    del K
    torch.cuda.empty_cache()
