"""Smallest distributed-SMO rehearsal runs (one GPU), printed step by step, checked against the
single-GPU solve: run before the full GPU tests so a fault shows up on a tiny case."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.parallel.dsmo import DsmoGroup  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

cases = [(int(a), int(b)) for a, b in (c.split("x") for c in (sys.argv[1] if len(sys.argv) > 1 else "3000x1").split(","))]
for n, P in cases:
    tr = synthetic_mnist(n, seed=31).compact()
    dev = torch.device("cuda:0")
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, tr.d)
    K, path = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    a = torch.zeros(n, dtype=torch.float64, device=dev)
    r, t1 = D.smo(K, yd, a, SVMParams(), n=n, trace_cap=100000)
    del K
    print(f"n={n} P={P}: single {r.iterations} it b={r.b!r}", flush=True)
    g = DsmoGroup(P, rehearsal=True, timeout_s=30)
    print(f"n={n} P={P}: group created", flush=True)
    out = g.fit(tr.X, tr.y, SVMParams(), trace_cap=100000)
    same = out["iterations"] == r.iterations and out["b"] == r.b and np.array_equal(out["trace"], t1) and \
        np.array_equal(out["alpha"], a.cpu().numpy())
    print(f"n={n} P={P}: dsmo {out['iterations']} it b={out['b']!r} shape={out['shape']} "
          f"timings={out['timings_ms']} identical={same}", flush=True)
    g.close()
    if not same:
        sys.exit(3)
