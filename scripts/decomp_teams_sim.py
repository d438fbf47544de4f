#!/usr/bin/env python3
"""Host simulation of the working-set decomposition with P concurrent teams (design study).

The device solver (csrc/hip/decomp.hip) solves ONE working set per outer iteration in one workgroup.
This script runs the same outer loop on the host (float64 numpy, kernel values exp(-gamma d^2) from
the scaled rows -- not the device's exact-integer values, so counts are close, not identical) with
P teams: the selection's candidates are dealt into P disjoint working sets, every team solves its own
set from the same (alpha, f), and the P steps are combined by the exact minimiser of the dual over
lambda in [0, 1]^P (the steps are feasible one by one, so every such combination is).  It prints
outer iterations, the critical path of inner iterations (sum over outer iterations of the slowest
team) and the combine's lambdas, for the design decisions in README "Concurrent working sets".

    python scripts/decomp_teams_sim.py --n 60000 --teams 1,2,4,8 --q 1024
"""
from __future__ import annotations

import argparse
import time

import numpy as np

from svm355.utils.data import MinMaxScaler, synthetic_mnist

C, GAMMA, TAU, EPS = 10.0, 0.00125, 1e-5, 1e-12


class Kern:
    def __init__(self, X):
        self.X = X
        self.sq = np.einsum("ij,ij->i", X, X)

    def block(self, I, J):
        d = self.sq[I][:, None] + self.sq[J][None, :] - 2.0 * (self.X[I] @ self.X[J].T)
        K = np.exp(-GAMMA * np.maximum(d, 0.0))
        K[np.asarray(I)[:, None] == np.asarray(J)[None, :]] = 1.0
        return K


def sets(a, y):
    below, above = a < C - EPS, a > EPS
    hi = ((y == 1) & below) | ((y == -1) & above)
    lo = ((y == 1) & above) | ((y == -1) & below)
    return hi, lo


def inner(Kw, y, a, f, tau_in, max_inner):
    """The device inner solve (first-order i, second-order j, reference clip / update arithmetic)."""
    a = a.copy()
    f = f.copy()
    it = 0
    while True:
        hi, lo = sets(a, y)
        if not hi.any() or not lo.any():
            break
        fh = np.where(hi, f, np.inf)
        ih = int(np.argmin(fh))
        bh = fh[ih]
        bl = np.max(np.where(lo, f, -np.inf))
        if bl <= bh + 2 * tau_in or it >= max_inner:
            break
        at = 2.0 - 2.0 * Kw[ih]
        at = np.where(at <= 0, EPS, at)
        gain = np.where(lo & (f > bh), -((f - bh) ** 2) / at, np.inf)
        il = int(np.argmin(gain))
        K12 = Kw[ih, il]
        yh, yl = y[ih], y[il]
        ah, al = a[ih], a[il]
        s = yh * yl
        eta = 2.0 - 2.0 * K12
        if s == -1:
            U, V = max(0.0, al - ah), min(C, C + al - ah)
        else:
            U, V = max(0.0, al + ah - C), min(C, al + ah)
        if not U <= V + 1e-12 or eta <= EPS:
            break
        aln = min(max(al + yl * (bh - f[il]) / eta, U), V)
        ahn = ah + s * (al - aln)
        f += (ahn - ah) * yh * Kw[ih] + (aln - al) * yl * Kw[il]
        a[ih], a[il] = ahn, aln
        it += 1
    return a, it


def inner_shrunk(Kw, y, a, f, tau_in, max_inner, na, stats):
    """Two-tier inner solve: the pair updates run on an active subset A of at most `na` points of W
    (the na/2 most violating of I_high and of I_low), to A's own gap <= 2 tau_in; then W's f is brought
    up to date from K(W, A) and W's gap checked -- another round on a fresh A while it is open."""
    a = a.copy()
    f = f.copy()
    it = 0
    m = len(a)
    while True:
        hi, lo = sets(a, y)
        if not hi.any() or not lo.any():
            break
        fh = np.where(hi, f, np.inf)
        fl = np.where(lo, f, -np.inf)
        bh, bl = fh.min(), fl.max()
        if bl <= bh + 2 * tau_in or it >= max_inner:
            break
        stats["rounds"] += 1
        oh = np.argsort(fh, kind="stable")[: na // 2]
        ol = np.argsort(-fl, kind="stable")[: na // 2]
        A = np.unique(np.concatenate([oh[np.isfinite(fh[oh])], ol[np.isfinite(fl[ol])]]))
        if len(A) > na:
            A = A[:na]
        KA = Kw[np.ix_(A, A)]
        aA, itA = inner(KA, y[A], a[A], f[A], tau_in, max_inner - it)
        d = (aA - a[A]) * y[A]
        a[A] = aA
        f += Kw[:, A] @ d
        it += itA
        stats["sizes"].append(len(A))
        if itA == 0:
            break
    return a, it


def box_qp(g, M, iters=200):
    """min g.l + l'Ml/2 over l in [0, 1]^P by coordinate descent from the better of all-ones and the
    best single team (convex: monotone decrease)."""
    P = len(g)
    obj = lambda l: g @ l + 0.5 * l @ M @ l  # noqa: E731
    cands = [np.ones(P)] + [np.eye(P)[p] for p in range(P)]
    lam = min(cands, key=obj).copy()
    for _ in range(iters):
        for p in range(P):
            if M[p, p] <= 0:
                continue
            r = g[p] + M[p] @ lam - M[p, p] * lam[p]
            lam[p] = min(1.0, max(0.0, -r / M[p, p]))
    return lam, obj(lam)


def select(f, a, y, NB, per, T):
    hi, lo = sets(a, y)
    H, L = [], []
    n = len(f)
    for b in range(NB):
        s, e = b * per, min(n, (b + 1) * per)
        fh = np.where(hi[s:e], f[s:e], np.inf)
        fl = np.where(lo[s:e], f[s:e], -np.inf)
        oh = np.argsort(fh, kind="stable")[:T]
        ol = np.argsort(-fl, kind="stable")[:T]
        H.append([(s + i, k) if np.isfinite(fh[i]) else (-1, k) for k, i in enumerate(oh)])
        L.append([(s + i, k) if np.isfinite(fl[i]) else (-1, k) for k, i in enumerate(ol)])
    return H, L


def run(X, y, teams, q, deal, combine, log, shrink=0, a0=None, tau_frac=0.1, per_outer=None):
    n = len(y)
    K = Kern(X)
    NB0 = max((n + 4095) // 4096, min(64, (n + 63) // 64))
    NB = (NB0 + 7) // 8 * 8
    per = (n + NB - 1) // NB
    T = max(1, q // (2 * NB))  # per team, per block, per side
    a = np.zeros(n) if a0 is None else a0.astype(np.float64).copy()
    f = -y.astype(np.float64)
    if a0 is not None:
        nz = np.flatnonzero(a != 0)
        f += K.block(np.arange(n), nz) @ (a[nz] * y[nz])
    outer = crit = total = 0
    lams = []
    sstats = {"rounds": 0, "sizes": []}
    yf = y.astype(np.float64)
    while True:
        H, L = select(f, a, y, NB, per, T * teams)
        hi, lo = sets(a, y)
        bh = np.min(np.where(hi, f, np.inf))
        bl = np.max(np.where(lo, f, -np.inf))
        if bl <= bh + 2 * TAU:
            break
        tau_in = max(TAU, tau_frac * (bl - bh))
        owner = {}
        # claims in per-block rank order (both sides of rank k before rank k + 1): the blocks' first
        # picks -- among them the global maximal violating pair -- all land in team 0
        recs = sorted((k, s, b, i) for s, side in enumerate((H, L)) for b, lst in enumerate(side)
                      for i, k in lst if i >= 0)
        for k, s, b, i in recs:
            p = k % teams if deal == "rank" else (b % teams)
            owner.setdefault(i, p)
        Ws = [np.array(sorted(i for i, p in owner.items() if p == t), dtype=np.int64) for t in range(teams)]
        steps = []
        its = []
        for W in Ws:
            if len(W) < 2:
                steps.append((W, np.zeros(len(W))))
                its.append(0)
                continue
            Kw = K.block(W, W)
            if shrink:
                an, it = inner_shrunk(Kw, y[W], a[W], f[W], tau_in, 20 * len(W), shrink, sstats)
            else:
                an, it = inner(Kw, y[W], a[W], f[W], tau_in, 20 * len(W))
            steps.append((W, (an - a[W]) * yf[W]))
            its.append(it)
        outer += 1
        if per_outer is not None:
            per_outer.append((bl - bh, [len(W) for W in Ws], its))
        crit += max(its)
        total += sum(its)
        mv = [(W[c != 0], c[c != 0]) for W, c in steps]
        U = [K.block(np.arange(n), W) @ c if len(W) else np.zeros(n) for W, c in mv]
        P = len(mv)
        g = np.array([f[W] @ c for W, c in mv])
        M = np.array([[mv[qq][1] @ U[p][mv[qq][0]] for qq in range(P)] for p in range(P)])
        M = 0.5 * (M + M.T)
        if combine == "qp" and P > 1:
            lam, _ = box_qp(g, M)
        else:
            lam = np.ones(P)
        lams.append(lam)
        for p, (W, c) in enumerate(mv):
            a[W] += lam[p] * c * yf[W]
            f += lam[p] * U[p]
        np.clip(a, 0.0, C, out=a)
        if log:
            print(f"  outer {outer}: gap {bl - bh:.3e} m {[len(W) for W in Ws]} inner {its} "
                  f"lambda {np.round(lam, 3).tolist()}", flush=True)
        if total > 100000:
            break
    sv = int(np.sum(a > 1e-8))
    run.alpha = a
    return outer, crit, total, sv, (bh + bl) / 2, sstats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--teams", default="1,2,4,8")
    ap.add_argument("--q", type=int, default=1024, help="working-set size per team")
    ap.add_argument("--deal", choices=["rank", "block"], default="rank")
    ap.add_argument("--combine", choices=["qp", "sum"], default="qp")
    ap.add_argument("--log", action="store_true")
    ap.add_argument("--shrink", type=int, default=0, help="two-tier inner solve on active subsets of this size")
    a = ap.parse_args()
    tr = synthetic_mnist(a.n, seed=2024)
    X = MinMaxScaler().fit_transform(tr.X)
    for P in [int(t) for t in a.teams.split(",")]:
        t0 = time.time()
        outer, crit, total, sv, b, ss = run(X, tr.y, P, a.q, a.deal, a.combine, a.log, a.shrink)
        print(f"n={a.n} teams={P} q={a.q} deal={a.deal} combine={a.combine}: outer {outer}, critical-path inner "
              f"iterations {crit}, all teams {total}, SVs {sv}, b {b:.7f} ({time.time() - t0:.0f} s)"
              + (f"; shrink {a.shrink}: {ss['rounds']} active-set rounds, mean size "
                 f"{np.mean(ss['sizes']):.0f}" if a.shrink else ""), flush=True)


if __name__ == "__main__":
    main()
