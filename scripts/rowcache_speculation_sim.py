"""How many passes over the quantised rows would a row cache that also fills SPECULATIVE rows on a
miss need?  A numpy first-order SMO (same selection and update as the oracle, lowest-index ties)
records every iteration's f; the replay counts miss events (each a full pass over the n rows) and
rows filled, for speculation from (a) the global top-B violators and (b) the workgroup-local
arg-min / arg-max candidates the persistent solver's exchange records already carry (slices of S
elements), capped at R rows per event.  Used to size the batched-fill experiment recorded in
profiles/r2_rowcache_batched_fill_ab.txt.

    python scripts/rowcache_speculation_sim.py 20000
"""
import sys, numpy as np
sys.path.insert(0, "/root/repo")
from svm355.ops import cpu as C
from svm355.utils.data import synthetic_mnist
n = int(sys.argv[1]); Cc, tau, eps = 10.0, 1e-5, 1e-12
tr = synthetic_mnist(n, seed=2024)
X = tr.X.astype(np.float64); mn, mx = X.min(0), X.max(0); r = mx - mn; r[r < 1e-12] = 1; X = (X - mn) / r
y = tr.y.astype(np.float64)
K = C.rbf_matrix(X, X, 0.00125, 8)
a = np.zeros(n); f = -y.copy()
pairs = []
for it in range(200000):
    up = ((y > 0) & (a < Cc - eps)) | ((y < 0) & (a > eps))
    low = ((y > 0) & (a > eps)) | ((y < 0) & (a < Cc - eps))
    fu = np.where(up, f, np.inf); fl = np.where(low, f, -np.inf)
    ih, il = int(np.argmin(fu)), int(np.argmax(fl))
    bh, bl = fu[ih], fl[il]
    if bl <= bh + 2 * tau: break
    pairs.append((ih, il, fu, fl))
    eta = K[ih, ih] + K[il, il] - 2 * K[ih, il]
    yh, yl = y[ih], y[il]; ah, al = a[ih], a[il]
    s = yh * yl
    if s < 0: U, V = max(0, al - ah), min(Cc, Cc + al - ah)
    else: U, V = max(0, al + ah - Cc), min(Cc, al + ah)
    al_new = min(max(al + yl * (bh - bl) / eta, U), V)
    ah_new = ah + s * (al - al_new)
    f += (ah_new - ah) * yh * K[ih] + (al_new - al) * yl * K[il]
    a[ih], a[il] = ah_new, al_new
T = len(pairs)
print(f"n={n} iterations {T} distinct rows {len(set([p[0] for p in pairs]) | set([p[1] for p in pairs]))}", flush=True)
for B in (0, 4, 8, 16, 32, 64):
    cached = set(); events = 0; filled = 0
    for ih, il, fu, fl in pairs:
        if ih in cached and il in cached: continue
        events += 1
        new = {ih, il} - cached
        if B:
            # speculative: the B/2 lowest f in I_up and B/2 highest f in I_low (current iterate)
            k = B // 2
            cu = np.argpartition(fu, k)[:k]; cl = np.argpartition(-fl, k)[:k]
            new |= set(int(x) for x in cu if np.isfinite(fu[x])) | set(int(x) for x in cl if np.isfinite(fl[x]))
        new -= cached
        filled += len(new); cached |= new
    print(f"B={B:3d}: miss events (passes over the rows) {events:6d}, rows filled {filled:6d}", flush=True)
# WG-local bests (what the exchange records already carry): slices of S elements
for S in (2048, 1024, 512):
    G = (n + S - 1) // S
    cached = set(); events = 0; filled = 0
    for ih, il, fu, fl in pairs:
        if ih in cached and il in cached: continue
        events += 1
        new = {ih, il}
        for g in range(G):
            sl = slice(g * S, min(n, (g + 1) * S))
            a1 = int(np.argmin(fu[sl])); b1 = int(np.argmax(fl[sl]))
            if np.isfinite(fu[sl][a1]): new.add(g * S + a1)
            if np.isfinite(fl[sl][b1]): new.add(g * S + b1)
        new -= cached
        filled += len(new); cached |= new
    print(f"WG-local bests, slice {S} (G={G}, <= {2*G} candidates): miss events {events:6d}, rows filled {filled:6d}", flush=True)
# capped batches: R-2 speculative rows from the WG-local bests, (a) in record order, (b) most violating first
for S, R in ((512, 32), (256, 32), (256, 16)):
    G = (n + S - 1) // S
    for mode in ("record-order", "by-value"):
        cached = set(); events = 0; filled = 0
        for ih, il, fu, fl in pairs:
            if ih in cached and il in cached: continue
            events += 1
            new = [x for x in (ih, il) if x not in cached]
            cands = []
            for g in range(G):
                sl = slice(g * S, min(n, (g + 1) * S))
                a1 = int(np.argmin(fu[sl])); b1 = int(np.argmax(fl[sl]))
                if np.isfinite(fu[sl][a1]): cands.append((fu[sl][a1], 0, g * S + a1))
                if np.isfinite(fl[sl][b1]): cands.append((-fl[sl][b1], 1, g * S + b1))
            if mode == "by-value":
                cands.sort(key=lambda c: c[0])
            for _, _, c in cands:
                if len(new) >= R: break
                if c not in cached and c not in new: new.append(c)
            filled += len(new); cached |= set(new)
        print(f"slice {S} G={G} R={R} {mode:12s}: miss events {events:6d}, rows filled {filled:6d}", flush=True)
