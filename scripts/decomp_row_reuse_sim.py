#!/usr/bin/env python3
"""How often the inner solve's two K(W, W) row loads per pair update (row i_high, then row j) name a row
loaded in the last few pair updates: LRU hit rates of an R-row on-chip row cache (design input for the
inner-solve latency chain).  Runs the host replica of the device solve
(scripts/decomp_teams_sim.py, one team) and records every pair's (i, j).

    python scripts/decomp_row_reuse_sim.py 60000
"""
import sys
from collections import OrderedDict

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import decomp_teams_sim as S  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402
from svm355.utils.data import MinMaxScaler  # noqa: E402

pairs = []  # per outer iteration: [(i, j), ...] in W positions
first_j = []  # per pair update: the second-order j is the first-order (maximal f in I_low) one
_inner = S.inner


ranks = []  # per outer iteration: W positions by violation at the start of the inner solve


def inner(Kw, y, a, f, tau_in, max_inner):
    rec = []
    hi0, lo0 = S.sets(a, y)
    bh0 = np.min(np.where(hi0, f, np.inf))
    bl0 = np.max(np.where(lo0, f, -np.inf))
    score = np.maximum(np.where(hi0, bl0 - f, -np.inf), np.where(lo0, f - bh0, -np.inf))
    ranks.append(np.argsort(-score, kind="stable"))
    a = a.copy()
    f = f.copy()
    it = 0
    while True:
        hi, lo = S.sets(a, y)
        if not hi.any() or not lo.any():
            break
        fh = np.where(hi, f, np.inf)
        ih = int(np.argmin(fh))
        bh = fh[ih]
        bl = np.max(np.where(lo, f, -np.inf))
        if bl <= bh + 2 * tau_in or it >= max_inner:
            break
        at = 2.0 - 2.0 * Kw[ih]
        at = np.where(at <= 0, S.EPS, at)
        gain = np.where(lo & (f > bh), -((f - bh) ** 2) / at, np.inf)
        il = int(np.argmin(gain))
        rec.append((ih, il))
        first_j.append(il == int(np.argmax(np.where(lo, f, -np.inf))))
        K12 = Kw[ih, il]
        yh, yl = y[ih], y[il]
        ah, al = a[ih], a[il]
        s = yh * yl
        eta = 2.0 - 2.0 * K12
        if s == -1:
            U, V = max(0.0, al - ah), min(S.C, S.C + al - ah)
        else:
            U, V = max(0.0, al + ah - S.C), min(S.C, al + ah)
        if not U <= V + 1e-12 or eta <= S.EPS:
            break
        aln = min(max(al + yl * (bh - f[il]) / eta, U), V)
        ahn = ah + s * (al - aln)
        f += (ahn - ah) * yh * Kw[ih] + (aln - al) * yl * Kw[il]
        a[ih], a[il] = ahn, aln
        it += 1
    pairs.append(rec)
    return a, it


S.inner = inner
n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
tr = synthetic_mnist(n, seed=2024)
X = MinMaxScaler().fit_transform(tr.X)
outer, crit, total, sv, b, _ = S.run(X, tr.y, 1, 1024, "rank", "qp", False)
print(f"n={n}: outer {outer} pair updates {total} b {b:.7f}; second-order j = first-order j in "
      f"{np.mean(first_j):.3f} of the pair updates")
for R in tuple(int(v) for v in sys.argv[2].split(",")) if len(sys.argv) > 2 else (4, 8, 12, 16, 18, 24, 32):
    hits = acc = hi_i = hi_j = 0
    for rec in pairs:  # the cache starts empty per outer iteration (a new K(W, W))
        lru = OrderedDict()
        for i, j in rec:
            for r, side in ((i, 0), (j, 1)):
                acc += 1
                if r in lru:
                    hits += 1
                    hi_i += side == 0
                    hi_j += side == 1
                    lru.move_to_end(r)
                else:
                    lru[r] = True
                    if len(lru) > R:
                        lru.popitem(last=False)
    print(f"R={R:3d} rows: hit rate {hits / acc:.3f} (row i {2 * hi_i / acc:.3f}, row j {2 * hi_j / acc:.3f})",
          flush=True)

# L2 warming design input: the rows an inner solve touches at all, and how many of them are among the
# P most violating W positions at its start (rows a kernel could load into the inner CU's L2 before it)
used = [len({r for p in rec for r in p}) for rec in pairs]
print(f"distinct rows per inner solve: mean {np.mean(used):.0f}, max {max(used)}; row loads per inner solve "
      f"{np.mean([2 * len(rec) for rec in pairs]):.0f}")
for P in (128, 192, 256, 320, 384, 512):
    cov = tot = 0
    for rec, rk in zip(pairs, ranks):
        u = {r for p in rec for r in p}
        cov += len(u & set(rk[:P].tolist()))
        tot += len(u)
    print(f"P={P:3d} most violating rows warmed: {cov / tot:.3f} of the first touches covered", flush=True)
