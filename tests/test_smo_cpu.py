"""L3 CPU oracle: exact reference semantics (main3.cpp:106-294, warm start mpi_svm_main3.cpp:155-290).

The oracle is compared against an independent pure-Python transcription of the reference loop
(bit-identical alphas and iteration count), against itself across thread counts, and against
scikit-learn's libsvm (same optimum within the stopping tolerance)."""
import math

import numpy as np
import pytest

from svm355 import SVMParams
from svm355.ops import cpu as C
from svm355.utils.data import MinMaxScaler


def py_reference_smo(X, y, C_=10.0, gamma=0.00125, tau=1e-5, eps=1e-12, max_iter=100000, alpha=None, wss=1):
    """Line-by-line transcription of SMO_train (main3.cpp:162-294), warm start if alpha given.
    wss=2: the second index is chosen by second-order gain (Fan, Chen & Lin 2005, WSS 2) among
    I_low points with f above b_high; i_high, the stop test and b stay first-order."""
    n, d = X.shape

    def kern(a, b):
        res = 0.0
        for k in range(d):
            res += (a[k] - b[k]) * (a[k] - b[k])
        return math.exp(-gamma * res)

    if alpha is None:
        alpha = [0.0] * n
        f = [-float(y[i]) for i in range(n)]
    else:
        alpha = list(alpha)
        f = []
        for i in range(n):
            s = 0.0
            for j in range(n):
                if alpha[j] == 0.0:
                    continue
                s += alpha[j] * y[j] * kern(X[j], X[i])
            f.append(s - float(y[i]))
    ihp = ilp = n
    Kh = [0.0] * n
    Kl = [0.0] * n
    num_iter = 1
    bh = bl = 0.0
    reason = None
    while True:
        ih, mn = n, math.inf
        il, mx = n, -math.inf
        for i in range(n):
            in_h = (y[i] == 1 and alpha[i] < C_ - eps) or (y[i] == -1 and alpha[i] > 0.0 + eps)
            in_l = (y[i] == 1 and alpha[i] > 0.0 + eps) or (y[i] == -1 and alpha[i] < C_ - eps)
            if in_h and f[i] < mn:
                mn, ih = f[i], i
            if in_l and f[i] > mx:
                mx, il = f[i], i
        if ih >= n or il >= n:
            reason = "no_candidate"
            break
        bh, bl = f[ih], f[il]
        if bl <= bh + 2.0 * tau:
            reason = "converged"
            break
        if ih != ihp:
            ihp = ih
            Kh = [kern(X[ih], X[j]) for j in range(n)]
        if wss == 2:
            jbest, gbest = n, math.inf
            for t in range(n):
                in_l = (y[t] == 1 and alpha[t] > 0.0 + eps) or (y[t] == -1 and alpha[t] < C_ - eps)
                if not in_l or not f[t] > bh:
                    continue
                bb = f[t] - bh
                at = Kh[ih] + 1.0 - 2.0 * Kh[t]  # K(t, t) = 1 for the RBF kernel
                if at <= 0.0:
                    at = eps
                g = -(bb * bb) / at
                if g < gbest:
                    gbest, jbest = g, t
            il, bl_upd = jbest, f[jbest]
        else:
            bl_upd = bl
        if il != ilp:
            ilp = il
            Kl = [kern(X[il], X[j]) for j in range(n)]
        s = y[ih] * y[il]
        eta = Kh[ih] + Kl[il] - 2.0 * Kh[il]
        ah, al = alpha[ih], alpha[il]
        if s == -1:
            U, V = max(0.0, al - ah), min(C_, C_ + al - ah)
        else:
            U, V = max(0.0, al + ah - C_), min(C_, al + ah)
        if not U <= V + 1e-12:
            reason = "infeasible"
            break
        if eta <= eps:
            reason = "nonpositive_eta"
            break
        aln = al + y[il] * (bh - bl_upd) / eta
        aln = min(aln, V)
        aln = max(aln, U)
        ahn = ah + s * (al - aln)
        dh, dl = ahn - ah, aln - al
        for i in range(n):
            f[i] += dh * y[ih] * Kh[i] + dl * y[il] * Kl[i]
        alpha[ih], alpha[il] = ahn, aln
        num_iter += 1
        if num_iter > max_iter:
            reason = "max_iter"
            break
    return np.array(alpha), num_iter, (bh + bl) / 2, reason


def _toy(n=70, d=6, seed=0, gamma_scale=1.0):
    rng = np.random.default_rng(seed)
    X = rng.integers(0, 256, size=(n, d)).astype(float)
    y = np.where(X[:, 0] + 0.5 * X[:, 1] + rng.normal(0, 40, n) > 190, 1, -1).astype(np.int32)
    return MinMaxScaler().fit_transform(X), y


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_oracle_bit_identical_to_python_transcription(seed):
    X, y = _toy(seed=seed)
    p = SVMParams(gamma=0.5)
    a, res, _ = C.smo_train(X, y, p)
    a_ref, it_ref, b_ref, reason = py_reference_smo(X, y.tolist(), gamma=0.5)
    assert res.iterations == it_ref
    assert res.stop_reason == reason
    np.testing.assert_array_equal(a, a_ref)
    assert res.b == b_ref


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_wss2_oracle_bit_identical_to_python_transcription(seed):
    X, y = _toy(seed=seed)
    p = SVMParams(gamma=0.5, wss=2)
    a, res, _ = C.smo_train(X, y, p)
    a_ref, it_ref, b_ref, reason = py_reference_smo(X, y.tolist(), gamma=0.5, wss=2)
    assert res.iterations == it_ref
    assert res.stop_reason == reason
    np.testing.assert_array_equal(a, a_ref)
    assert res.b == b_ref


def test_wss2_reaches_the_first_order_optimum_in_fewer_iterations(small_mnist):
    """Second-order selection changes the path, not the problem: same SVs (within 2), b within the
    stopping tolerance, fewer iterations, same result with any thread count."""
    tr, _ = small_mnist
    X = MinMaxScaler().fit_transform(tr.X[:600])
    y = tr.y[:600]
    a1, r1, _ = C.smo_train(X, y, SVMParams(n_threads=2))
    a2, r2, t2 = C.smo_train(X, y, SVMParams(n_threads=2, wss=2), trace_cap=100000)
    a2s, r2s, t2s = C.smo_train(X, y, SVMParams(n_threads=1, wss=2), trace_cap=100000)
    assert r1.stop_reason == r2.stop_reason == "converged"
    assert r2.iterations < r1.iterations
    sv1, sv2 = set(np.flatnonzero(a1 > 1e-8).tolist()), set(np.flatnonzero(a2 > 1e-8).tolist())
    assert len(sv1 ^ sv2) <= 2
    assert abs(r1.b - r2.b) < 1e-4 * max(1.0, abs(r1.b))
    assert r2.iterations == r2s.iterations and r2.b == r2s.b
    np.testing.assert_array_equal(a2, a2s)
    np.testing.assert_array_equal(t2, t2s)


def test_warm_start_bit_identical_to_python_transcription():
    X, y = _toy(seed=5)
    p = SVMParams(gamma=0.5)
    a_cold, _, _ = C.smo_train(X, y, p, trace_cap=0)
    # Perturb a converged solution (keeps feasibility: scale both classes' alphas equally).
    a0 = a_cold * 0.5
    a, res, _ = C.smo_train(X, y, p, alpha=a0, warm=True)
    a_ref, it_ref, b_ref, _ = py_reference_smo(X, y.tolist(), gamma=0.5, alpha=a0.tolist())
    assert res.iterations == it_ref
    np.testing.assert_array_equal(a, a_ref)
    assert res.b == b_ref


def test_threads_do_not_change_results(small_mnist):
    tr, _ = small_mnist
    X = MinMaxScaler().fit_transform(tr.X[:600])
    y = tr.y[:600]
    a1, r1, t1 = C.smo_train(X, y, SVMParams(n_threads=1), trace_cap=100000)
    a8, r8, t8 = C.smo_train(X, y, SVMParams(n_threads=8), trace_cap=100000)
    assert r1.iterations == r8.iterations
    np.testing.assert_array_equal(a1, a8)
    np.testing.assert_array_equal(t1, t8)
    assert r1.b == r8.b


def test_gram_path_matches_row_path(small_mnist):
    tr, _ = small_mnist
    X = MinMaxScaler().fit_transform(tr.X[:400])
    y = tr.y[:400]
    p = SVMParams(n_threads=4)
    K = C.rbf_matrix(X, X, p.gamma)
    a1, r1, t1 = C.smo_train(X, y, p, trace_cap=100000)
    a2, r2, t2 = C.smo_train_gram(K, y, p, trace_cap=100000)
    assert r1.iterations == r2.iterations
    np.testing.assert_array_equal(a1, a2)
    np.testing.assert_array_equal(t1, t2)


def test_first_iteration_tie_break_is_lowest_index():
    # f = -y initially: every y=+1 ties at -1 (I_high), every y=-1 ties at +1 (I_low).
    X, y = _toy(seed=3)
    _, _, trace = C.smo_train(X, y, SVMParams(gamma=0.5), trace_cap=1)
    assert trace[0, 0] == np.flatnonzero(y == 1)[0]
    assert trace[0, 1] == np.flatnonzero(y == -1)[0]


def test_warm_start_from_zero_equals_cold(small_mnist):
    tr, _ = small_mnist
    X = MinMaxScaler().fit_transform(tr.X[:300])
    y = tr.y[:300]
    p = SVMParams(n_threads=4)
    a1, r1, _ = C.smo_train(X, y, p)
    a2, r2, _ = C.smo_train(X, y, p, alpha=np.zeros(300), warm=True)
    np.testing.assert_array_equal(a1, a2)
    assert r1.iterations == r2.iterations


def test_max_iter_stop_and_counter_semantics():
    X, y = _toy(seed=4)
    a, res, trace = C.smo_train(X, y, SVMParams(gamma=0.5, max_iter=5), trace_cap=100)
    assert res.stop_reason == "max_iter"
    assert res.iterations == 6  # num_iter starts at 1 and the check is num_iter > max_iter
    assert trace.shape == (5, 2)


def test_single_class_no_candidate():
    X, _ = _toy(seed=0, n=20)
    y = np.ones(20, dtype=np.int32)
    a, res, _ = C.smo_train(X, y, SVMParams(gamma=0.5))
    assert res.stop_reason == "no_candidate"
    assert np.all(a == 0)


def test_kkt_and_constraints_at_solution(small_mnist):
    tr, _ = small_mnist
    X = MinMaxScaler().fit_transform(tr.X[:500])
    y = tr.y[:500]
    p = SVMParams(n_threads=4)
    a, res, _ = C.smo_train(X, y, p)
    assert res.stop_reason == "converged"
    assert abs(np.dot(a, y)) < 1e-9 * max(1.0, a.sum())
    assert a.min() >= 0 and a.max() <= p.C
    K = C.rbf_matrix(X, X, p.gamma)
    f = K @ (a * y) - y
    eps = p.eps
    up = ((y == 1) & (a < p.C - eps)) | ((y == -1) & (a > eps))
    low = ((y == 1) & (a > eps)) | ((y == -1) & (a < p.C - eps))
    assert f[low].max() <= f[up].min() + 2 * p.tau + 1e-9


def test_matches_sklearn_libsvm(small_mnist):
    sk = pytest.importorskip("sklearn.svm")
    tr, te = small_mnist
    sc = MinMaxScaler().fit(tr.X)
    X = sc.transform(tr.X)
    p = SVMParams(n_threads=4, tau=1e-6)
    a, res, _ = C.smo_train(X, tr.y, p)
    m = sk.SVC(C=p.C, kernel="rbf", gamma=p.gamma, tol=1e-6, shrinking=False).fit(X, tr.y)
    ours = set(np.flatnonzero(a > 1e-8).tolist())
    theirs = set(m.support_.tolist())
    assert len(ours ^ theirs) <= max(2, len(ours) // 100)
    # libsvm decision = sum a y K + rho_sklearn ; ours = sum a y K - b
    assert abs(-m.intercept_[0] - res.b) < 1e-3 * max(1.0, abs(res.b))
    dec = C.decision(X[a > 1e-8], tr.y[a > 1e-8], a[a > 1e-8], sc.transform(te.X), p.gamma, res.b)
    agree = np.mean(np.sign(dec) == np.sign(m.decision_function(sc.transform(te.X))))
    assert agree > 0.995


def test_decision_matches_numpy(small_mnist):
    tr, te = small_mnist
    sc = MinMaxScaler().fit(tr.X)
    Xs = sc.transform(tr.X[:50])
    Xq = sc.transform(te.X[:30])
    rng = np.random.default_rng(0)
    al = rng.uniform(0, 10, 50)
    ys = tr.y[:50]
    d2 = ((Xq[:, None, :] - Xs[None, :, :]) ** 2).sum(-1)
    ref = np.exp(-0.00125 * d2) @ (al * ys) - 0.3
    np.testing.assert_allclose(C.decision(Xs, ys, al, Xq, 0.00125, 0.3), ref, rtol=1e-12, atol=1e-12)
