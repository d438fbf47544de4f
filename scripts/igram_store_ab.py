"""Exact-integer Gram at n = 60000: nontemporal (shipped) vs plain stores (SVM355_IGRAM_STORE=plain,
read per launch), alternating rounds, each Gram right after an XCD-local 60k SMO (as in a bench fit)
and back-to-back; identical values required."""
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
n = 60000
tr = synthetic_mnist(n, seed=2024)
Xd = D.upload_rows(tr.compact().X, dev)
mn, mx, sqn = D.minmax_scale_(Xd, 784)
yd = torch.from_numpy(tr.y).to(dev)
K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
ref = K[::997].clone()
times = {(m, c): [] for m in ("nt", "plain") for c in ("after_smo", "b2b")}
for rnd in range(4):
    for m in ("nt", "plain"):
        if m == "plain":
            os.environ["SVM355_IGRAM_STORE"] = "plain"
        else:
            os.environ.pop("SVM355_IGRAM_STORE", None)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        D.smo(K, yd, a, SVMParams(), n=n)  # the one-XCD solve a bench fit runs before its next Gram
        for c in ("after_smo", "b2b"):
            torch.cuda.synchronize()
            t = time.perf_counter()
            K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, out=K)
            torch.cuda.synchronize()
            times[(m, c)].append((time.perf_counter() - t) * 1e3)
            assert torch.equal(K[::997], ref), m
    print(f"round {rnd} done", flush=True)
for k, v in times.items():
    print(f"n={n} stores {k[0]:5s} {k[1]:9s}: best {min(v):.2f} ms  median {statistics.median(v):.2f} ms", flush=True)
