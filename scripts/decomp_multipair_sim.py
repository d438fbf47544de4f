#!/usr/bin/env python3
"""Chain iterations of the decomposition inner solve with 1, 2 or 3 pair updates per iteration (design
input for a third pair).  Host replica of the device solve (scripts/decomp_teams_sim.py, one team) with
the inner solve replaced: every iteration selects i = argmin f over I_high and j by the second-order gain
(pair 1); pair 2 (ws_inner_kernel<..., DP>, decomp_cpu.cpp inner_wss = 3) takes i2 = the best I_high
candidate of the waves other than i's and j2 = the first-order j; pair 3 (not implemented on the device)
takes i3 = the best I_high candidate of the waves holding neither i nor i2 and j3 = the best I_low
candidate of the waves other than j2's.  Pairs 2 and 3 apply, in order, if still violating, disjoint
from the pairs before them and feasible.  The wave of W position k is (k mod 512) / 128 (256 threads x
4 points).

    python scripts/decomp_multipair_sim.py 60000 1,2,3
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import decomp_teams_sim as S  # noqa: E402
from svm355.utils.data import MinMaxScaler, synthetic_mnist  # noqa: E402

NPAIR = 1
J2_SECOND = False  # SIM_J2=second: the second pair's j by i2's second-order gain (not the first-order j)
stats = {"chain": 0, "pairs": 0}


def wave_best(vals, mask, waves, excl, want_min):
    """(position, value) of the best masked entry over the waves not in excl (lowest position on ties)."""
    ok = mask & ~np.isin(waves, list(excl))
    if not ok.any():
        return -1
    return int(np.argmin(np.where(ok, vals, np.inf)) if want_min else np.argmax(np.where(ok, vals, -np.inf)))


def pair_update(Kw, y, a, f, i, j, tau_in, need_violation):
    if i < 0 or j < 0 or i == j:
        return False
    if need_violation and not f[j] > f[i] + 2 * tau_in:
        return False
    yh, yl = y[i], y[j]
    ah, al = a[i], a[j]
    s = yh * yl
    eta = 2.0 - 2.0 * Kw[i, j]
    if s == -1:
        U, V = max(0.0, al - ah), min(S.C, S.C + al - ah)
    else:
        U, V = max(0.0, al + ah - S.C), min(S.C, al + ah)
    if not U <= V + 1e-12 or eta <= S.EPS:
        return None if not need_violation else False
    aln = min(max(al + yl * (f[i] - f[j]) / eta, U), V)
    ahn = ah + s * (al - aln)
    f += (ahn - ah) * yh * Kw[i] + (aln - al) * yl * Kw[j]
    a[i], a[j] = ahn, aln
    return True


def inner(Kw, y, a, f, tau_in, max_inner):
    a = a.copy()
    f = f.copy()
    m = len(a)
    waves = (np.arange(m) % 512) // 128
    it = 0
    while True:
        hi, lo = S.sets(a, y)
        if not hi.any() or not lo.any():
            break
        fh = np.where(hi, f, np.inf)
        ih = int(np.argmin(fh))
        bh = fh[ih]
        fl = np.where(lo, f, -np.inf)
        bl = np.max(fl)
        if bl <= bh + 2 * tau_in or it >= max_inner:
            break
        at = 2.0 - 2.0 * Kw[ih]
        at = np.where(at <= 0, S.EPS, at)
        gain = np.where(lo & (f > bh), -((f - bh) ** 2) / at, np.inf)
        il = int(np.argmin(gain))
        j_first = int(np.argmax(fl))
        # candidates of the later pairs come from the same selection (before any update)
        i2 = wave_best(f, hi, waves, {waves[ih]}, True) if NPAIR >= 2 else -1
        if J2_SECOND and i2 >= 0:  # j2 by the second-order gain of i2's row (same snapshot of f)
            at2 = 2.0 - 2.0 * Kw[i2]
            at2 = np.where(at2 <= 0, S.EPS, at2)
            g2 = np.where(lo & (f > f[i2]), -((f - f[i2]) ** 2) / at2, np.inf)
            j_first = int(np.argmin(g2)) if np.isfinite(g2).any() else j_first
        i3 = wave_best(f, hi, waves, {waves[ih]} | ({waves[i2]} if i2 >= 0 else set()), True) if NPAIR >= 3 else -1
        j3 = wave_best(f, lo, waves, {waves[j_first]}, False) if NPAIR >= 3 else -1
        r = pair_update(Kw, y, a, f, ih, il, tau_in, False)
        if r is None:
            break
        stats["pairs"] += 1
        used = {ih, il}
        if NPAIR >= 2 and i2 not in used and j_first not in used:
            if pair_update(Kw, y, a, f, i2, j_first, tau_in, True):
                stats["pairs"] += 1
                used |= {i2, j_first}
        if NPAIR >= 3 and i3 >= 0 and j3 >= 0 and i3 not in used and j3 not in used:
            if pair_update(Kw, y, a, f, i3, j3, tau_in, True):
                stats["pairs"] += 1
        it += 1
        stats["chain"] += 1
    return a, it


S.inner = inner
J2_SECOND = __import__("os").environ.get("SIM_J2") == "second"
n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
tr = synthetic_mnist(n, seed=2024)
X = MinMaxScaler().fit_transform(tr.X)
for NPAIR in (int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1,2,3").split(",")):
    stats.update(chain=0, pairs=0)
    outer, crit, total, sv, b, _ = S.run(X, tr.y, 1, 1024, "rank", "qp", False)
    print(f"n={n} pairs/iteration <= {NPAIR}: outer {outer} chain iterations {stats['chain']} pair updates "
          f"{stats['pairs']} SVs {sv} b {b:.7f}", flush=True)
