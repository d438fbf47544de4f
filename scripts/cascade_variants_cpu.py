"""Can a cascade variant beat the one-SMO trainer?  CPU-oracle study of iteration counts (no timing).

    python scripts/cascade_variants_cpu.py N        # synthetic MNIST, N rows, the headline C / gamma / tau

For P = 2, 4, 8 partitions (the layer the P GPUs would solve in parallel) this reports:
  * the full problem's cold first-order SMO (the single-GPU trainer's trajectory);
  * "warm polish": the P local solutions concatenated (a feasible point: every partition keeps
    sum(alpha * y) = 0) warm-start one SMO over all N rows;
  * "KKT star": rank 0 solves the union U of the local SVs (cold, or warm from the local alphas),
    then the exact global KKT test over all N rows (f = K[:, SV] (alpha y) - y, the solver's own
    b_low <= b_high + 2 tau rule); violators join U and the solve repeats warm.
The serial critical path of each variant is (slowest local solve) + (rank-0 solves), in SMO
iterations; the trainer's is its own count.  Result (profiles/r2_cascade_variants_cpu.txt): every
variant needs as many or more rank-0 iterations than the whole problem, so no cascade that ends in
a rank-0 solve over the candidate SVs can beat the single-GPU trainer at this size.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import cpu as C  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
tr = synthetic_mnist(n, seed=2024)
X = tr.X.astype(np.float64)
mn, mx = X.min(0), X.max(0)
rng = mx - mn
rng[rng < 1e-12] = 1.0
X = (X - mn) / rng
y = tr.y.astype(np.int32)
p = SVMParams(n_threads=8)
t0 = time.time()
K = C.rbf_matrix(X, X, p.gamma, 8)
print(f"n={n}: Gram {time.time() - t0:.1f} s", flush=True)
a0, r0, _ = C.smo_train_gram(K, y, p)
sv0 = set(np.flatnonzero(a0 > 0).tolist())
print(f"single SMO: iterations={r0.iterations} b={r0.b:.9f} n_sv={len(sv0)}", flush=True)


def solve_on(U, alpha=None):
    U = np.asarray(sorted(U))
    aU, rU, _ = C.smo_train_gram(np.ascontiguousarray(K[np.ix_(U, U)]), y[U], p,
                                 alpha=None if alpha is None else alpha[U], warm=alpha is not None)
    a = np.zeros(n)
    a[U] = aU
    return a, rU


def violators(a):
    f = K[:, a > 0] @ (a[a > 0] * y[a > 0]) - y
    up = ((y == 1) & (a < p.C)) | ((y == -1) & (a > 0))
    low = ((y == 1) & (a > 0)) | ((y == -1) & (a < p.C))
    bup, blow = f[up].min(), f[low].max()
    if blow <= bup + 2 * p.tau:
        return set()
    return set(np.flatnonzero((up & (f < blow - 2 * p.tau)) | (low & (f > bup + 2 * p.tau))).tolist())


def tag(a):
    sv = set(np.flatnonzero(a > 0).tolist())
    return f"n_sv={len(sv)} symdiff_vs_single={len(sv ^ sv0)}"


for P in (2, 4, 8):
    a = np.zeros(n)
    loc = 0
    for r in range(P):
        lo, hi = r * n // P, (r + 1) * n // P
        ap, rp, _ = C.smo_train_gram(np.ascontiguousarray(K[lo:hi, lo:hi]), y[lo:hi], p)
        a[lo:hi] = ap
        loc = max(loc, rp.iterations)
    U0 = set(np.flatnonzero(a > 0).tolist())
    aw, rw, _ = C.smo_train_gram(K, y, p, alpha=a, warm=True)
    print(f"P={P}: slowest local solve {loc} it, |U|={len(U0)} | warm polish over all rows: {rw.iterations} it, "
          f"b={rw.b:.9f} {tag(aw)} -> critical path {loc + rw.iterations} it", flush=True)
    for warm in (False, True):
        U = set(U0)
        am, rm = solve_on(U, a if warm else None)
        its = [rm.iterations]
        for _ in range(6):
            v = violators(am) - U
            if not v:
                break
            U |= v
            am, rm = solve_on(U, am)
            its.append(rm.iterations)
        print(f"      KKT star ({'warm' if warm else 'cold'} first merge): rank-0 solves {its} it, final |U|={len(U)}, "
              f"b={rm.b:.9f} {tag(am)} -> critical path {loc + sum(its)} it", flush=True)
