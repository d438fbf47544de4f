"""Probe: does a full 60k solve warm-started from the concatenated per-partition solutions need
fewer SMO iterations than the cold solve?  (Each partition's solve keeps sum(y*alpha) = 0, so the
concatenation is a feasible point of the full dual.)  One MI355X, partitions solved one by one."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from svm355.ops import device as D  # noqa: E402
from svm355.utils.config import SVMParams  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
dev = torch.device("cuda", 0)
tr = synthetic_mnist(n, seed=2024).compact()
p = SVMParams()
Xd = D.upload_rows(tr.X, dev)
yd = torch.from_numpy(tr.y).to(dev)
mn, mx, sqn = D.minmax_scale_(Xd, tr.X.shape[1])


def solve(X, s, y, a0=None):
    a = torch.zeros(X.shape[0], dtype=torch.float64, device=dev) if a0 is None else a0.clone()
    torch.cuda.synchronize()
    t = time.perf_counter()
    r, tm = D.train(X, s, y, a, p, warm=a0 is not None, mn=mn, mx=mx)
    torch.cuda.synchronize()
    return a, r, (time.perf_counter() - t) * 1e3, tm


a_cold, r_cold, ms_cold, tm = solve(Xd, sqn, yd)
sv_cold = set(torch.nonzero(a_cold > p.sv_tol).flatten().tolist())
print(f"cold n={n}: it={r_cold.iterations} b={r_cold.b:.10f} nsv={len(sv_cold)} {ms_cold:.1f} ms {tm}", flush=True)
for P in (2, 4, 8, 16):
    ch = (n + P - 1) // P
    parts, its, mss = [], [], []
    for r in range(P):
        lo, hi = r * ch, min(n, (r + 1) * ch)
        a, rr, ms, _ = solve(Xd[lo:hi].contiguous(), sqn[lo:hi].contiguous(), yd[lo:hi].contiguous())
        parts.append(a)
        its.append(rr.iterations)
        mss.append(ms)
    a0 = torch.cat(parts)
    a_w, r_w, ms_w, tm_w = solve(Xd, sqn, yd, a0)
    sv_w = set(torch.nonzero(a_w > p.sv_tol).flatten().tolist())
    nsv0 = int((a0 > p.sv_tol).sum())
    print(f"P={P}: local it max {max(its)} (sum {sum(its)}) max ms {max(mss):.1f} | seed nsv {nsv0} | warm full it={r_w.iterations} "
          f"b={r_w.b:.10f} nsv={len(sv_w)} symdiff={len(sv_w ^ sv_cold)} {ms_w:.1f} ms {tm_w}", flush=True)
