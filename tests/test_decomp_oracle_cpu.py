"""CPU oracle of the working-set decomposition solver (csrc/core/decomp_cpu.cpp).

On the GPU the oracle is compared with the device solver bit for bit (tests/test_gpu_decomp_oracle.py).
Here, on the CPU, it is checked against the problem itself: the reference's stop test recomputed from
the final alphas, the pairwise CPU oracle's support vectors on the same kernel matrix, and the
internal consistency of its per-outer-iteration trace (moved columns vs alpha, f vs K (alpha y) - y)."""
import numpy as np
import pytest

from svm355 import SVMParams
from svm355.ops import cpu as C
from svm355.utils.data import MinMaxScaler, synthetic_mnist


def _problem(n, seed):
    tr = synthetic_mnist(n, seed=seed)
    X = MinMaxScaler().fit_transform(tr.X)
    sq = np.einsum("ij,ij->i", X, X)
    K = np.exp(-0.00125 * np.maximum(sq[:, None] + sq[None, :] - 2.0 * X @ X.T, 0.0))
    np.fill_diagonal(K, 1.0)
    return K, tr.y.astype(np.int32)


def _gap(K, y, a, p):
    f = K @ (a * y) - y
    hi = ((y == 1) & (a < p.C - p.eps)) | ((y == -1) & (a > p.eps))
    lo = ((y == 1) & (a > p.eps)) | ((y == -1) & (a < p.C - p.eps))
    return f[lo].max() - f[hi].min()


@pytest.fixture(scope="module")
def prob2k():
    return _problem(2000, 11)


@pytest.mark.parametrize("q,inner_wss", [(1024, 3), (1024, 4), (1024, 2), (256, 3), (1024, 1)])
def test_oracle_meets_the_stop_test_with_the_pairwise_svs(prob2k, q, inner_wss):
    K, y = prob2k
    p = SVMParams(n_threads=4)
    a, r, st, _ = C.decomp_train_gram(K, y, p, q=q, inner_wss=inner_wss)
    assert r.stop_reason == "converged"
    assert st["outer_iterations"] >= 1 and r.iterations == st["inner_iterations"] + 1
    assert _gap(K, y, a, p) <= 2 * p.tau + 1e-9
    ref, rr, _ = C.smo_train_gram(K, y, p)
    np.testing.assert_array_equal(np.flatnonzero(a > p.sv_tol), np.flatnonzero(ref > p.sv_tol))
    assert abs(r.b - rr.b) <= 10 * p.tau
    assert np.all((a >= -1e-9) & (a <= p.C + 1e-9))  # the clip arithmetic rounds
    assert abs(float(a @ y)) < 1e-9 * max(1.0, a.sum())


def test_oracle_trace_is_consistent(prob2k):
    K, y = prob2k
    p = SVMParams(n_threads=4)
    a, r, st, tr = C.decomp_train_gram(K, y, p, trace_cap=200, snapshots=True)
    recs = tr.records()
    assert len(recs) == st["outer_iterations"]
    assert sum(x["inner"] for x in recs) == st["inner_iterations"]
    assert sum(x["moved"] for x in recs) == st["update_columns"]
    prev = np.zeros_like(a)
    for x in recs:
        W = x["W"]
        assert np.all(np.diff(W) > 0) and x["m"] <= st["working_set"]  # sorted, unique, within the capacity
        assert np.all(np.isin(x["cols"], W)) and np.all(np.diff(x["cols"]) > 0)
        d = x["alpha"] - prev
        moved = np.flatnonzero(d != 0)
        np.testing.assert_array_equal(moved, x["cols"])
        np.testing.assert_array_equal(d[moved] * y[moved], x["coef"])  # (a - a0) y, exactly
        act = ~np.isnan(x["f"])  # shrunk points carry NaN (their f is not part of the trajectory)
        np.testing.assert_allclose(x["f"][act], (K @ (x["alpha"] * y) - y)[act], rtol=0, atol=1e-10)
        bh, bl = x["bounds"]
        assert bl > bh + 2 * p.tau  # only running builds are recorded
        prev = x["alpha"]
    np.testing.assert_array_equal(prev, a)


def test_oracle_warm_start(prob2k):
    """Warm from its own solution the solve stops at once; warm from a feasible perturbation (a pair
    moved along y) it converges to the same support vectors."""
    K, y = prob2k
    p = SVMParams(n_threads=4)
    a, r, st, _ = C.decomp_train_gram(K, y, p)
    a2, r2, st2, _ = C.decomp_train_gram(K, y, p, alpha=a)
    assert st2["outer_iterations"] == 0 and r2.stop_reason == "converged"
    np.testing.assert_array_equal(a2, a)
    i = int(np.flatnonzero((a > 1e-3) & (a < p.C - 1e-3))[0])
    j = int(np.flatnonzero((y == y[i]) & (a > 1e-3) & (a < p.C - 1e-3) & (np.arange(len(y)) != i))[0])
    w = a.copy()
    delta = 0.5 * min(a[i], p.C - a[j])
    w[i] -= delta
    w[j] += delta  # same label: sum y alpha unchanged
    a3, r3, st3, _ = C.decomp_train_gram(K, y, p, alpha=w)
    assert r3.stop_reason == "converged" and st3["outer_iterations"] >= 1
    assert _gap(K, y, a3, p) <= 2 * p.tau + 1e-9
    np.testing.assert_array_equal(np.flatnonzero(a3 > p.sv_tol), np.flatnonzero(a > p.sv_tol))


AGGRESSIVE = {"SVM355_DECOMP_SHRINK": "1", "SVM355_DECOMP_SHRINK_START": "1", "SVM355_DECOMP_SHRINK_MARGIN": "0"}


@pytest.mark.parametrize("mode", ["default", "aggressive", "period3"])
def test_shrinking_keeps_the_stop_test_on_all_points(prob2k, monkeypatch, mode):
    """Shrinking (decomp_shrink.h): the solve on the active points, f recomputed from alpha when the active
    problem stops, the reference's stop test on all n points.  LIBSVM's rule every outer iteration
    (margin 0, "aggressive") shrinks points the solve needs again -- it must unshrink and still reach the
    unshrunk solve's support vectors; the trace shows NaN exactly for the points out of the active set,
    and only for points at a bound."""
    K, y = prob2k
    p = SVMParams(n_threads=4)
    ref, rr, _, _ = C.decomp_train_gram(K, y, p.replace(shrinking=False))
    if mode == "aggressive":
        for k, v in AGGRESSIVE.items():
            monkeypatch.setenv(k, v)
    q = p.replace(shrinking=3 if mode == "period3" else True)
    a, r, st, tr = C.decomp_train_gram(K, y, q, trace_cap=400, snapshots=True)
    assert r.stop_reason == "converged" and _gap(K, y, a, p) <= 2 * p.tau + 1e-9
    np.testing.assert_array_equal(np.flatnonzero(a > p.sv_tol), np.flatnonzero(ref > p.sv_tol))
    assert abs(r.b - rr.b) <= 10 * p.tau
    assert st["shrink_passes"] >= 1
    if mode == "aggressive":
        assert st["unshrinks"] >= 1 and st["min_active"] < len(y) // 2
    for x in tr.records():
        out = np.isnan(x["f"])
        ax = x["alpha"]
        free = (ax > p.eps) & (ax < p.C - p.eps)
        assert not np.any(out & free)  # only points at a bound are shrunk


def test_shrinking_off_is_the_unshrunk_trajectory(prob2k, monkeypatch):
    """shrinking=False and SVM355_DECOMP_SHRINK=0 are the same solve: no pass, nothing NaN."""
    K, y = prob2k
    p = SVMParams(n_threads=4, shrinking=False)
    a, r, st, tr = C.decomp_train_gram(K, y, p, trace_cap=400, snapshots=True)
    monkeypatch.setenv("SVM355_DECOMP_SHRINK", "0")
    a2, r2, st2, _ = C.decomp_train_gram(K, y, p.replace(shrinking=True))
    np.testing.assert_array_equal(a, a2)
    assert st["shrink_passes"] == st2["shrink_passes"] == 0 and st["min_active"] == len(y)
    assert not any(np.isnan(x["f"]).any() for x in tr.records())


def test_oracle_reports_the_real_working_set_capacity():
    """q below 2 x blocks: every block still gives its extreme pair, so the capacity is 2 NB, and
    stats say so (decomp_shape)."""
    K, y = _problem(6000, 12)
    p = SVMParams(n_threads=4)
    a, r, st, tr = C.decomp_train_gram(K, y, p, q=64, trace_cap=400)
    assert st["working_set"] == 128  # 64 blocks x 2 sides x 1 pick
    assert max(x["m"] for x in tr.records()) <= 128
    assert r.stop_reason == "converged" and _gap(K, y, a, p) <= 2 * p.tau + 1e-9


@pytest.mark.parametrize("world,shrink", [(1, "on"), (2, "on"), (4, "on"), (8, "on"), (2, "off"), (8, "off"),
                                          (2, "aggressive"), (8, "aggressive")])
def test_distributed_oracle_thread_ranks_are_bit_identical(prob2k, world, shrink, monkeypatch):
    """decomp.hip's world > 1 form on the CPU oracle: every rank owns 1/world of the blocks and of f,
    the candidate records are all-gathered (strict loopback), each rank keeps an alpha replica (the
    native side requires them all equal).  For world | 8 the block partition is the one-rank one, so
    alpha, b and the iteration counts equal the one-rank solve bit for bit -- also when the ranks shrink
    their own points and unshrink together (the build's bounds are global)."""
    if shrink == "aggressive":
        for k, v in AGGRESSIVE.items():
            monkeypatch.setenv(k, v)
    K, y = prob2k
    p = SVMParams(n_threads=2, shrinking=shrink != "off")
    a, r, st, _ = C.decomp_train_gram(K, y, p)
    a2, r2, st2 = C.decomp_train_gram_dist(K, y, p, world=world)
    np.testing.assert_array_equal(a2, a)
    assert r2.b == r.b and r2.iterations == r.iterations
    assert st2["outer_iterations"] == st["outer_iterations"] and st2["update_columns"] == st["update_columns"]


def test_distributed_oracle_other_world_converges(prob2k):
    """world = 3 does not divide 8: the blocks round to a multiple of 24 (another partition, another
    trajectory), and the solve still meets the stop test with the same support vectors."""
    K, y = prob2k
    p = SVMParams(n_threads=2)
    a, r, st = C.decomp_train_gram_dist(K, y, p, world=3)
    assert r.stop_reason == "converged" and _gap(K, y, a, p) <= 2 * p.tau + 1e-9
    ref, _, _, _ = C.decomp_train_gram(K, y, p)
    np.testing.assert_array_equal(np.flatnonzero(a > p.sv_tol), np.flatnonzero(ref > p.sv_tol))


def test_distributed_oracle_warm_start_is_bit_identical(prob2k):
    K, y = prob2k
    p = SVMParams(n_threads=2)
    a, _, _, _ = C.decomp_train_gram(K, y, p)
    w = a.copy()
    i = int(np.flatnonzero((a > 1e-3) & (a < p.C - 1e-3))[0])
    j = int(np.flatnonzero((y == y[i]) & (a > 1e-3) & (a < p.C - 1e-3) & (np.arange(len(y)) != i))[0])
    delta = 0.5 * min(a[i], p.C - a[j])
    w[i] -= delta
    w[j] += delta
    a1, r1, st1, _ = C.decomp_train_gram(K, y, p, alpha=w)
    a4, r4, st4 = C.decomp_train_gram_dist(K, y, p, world=4, alpha=w)
    np.testing.assert_array_equal(a4, a1)
    assert r4.b == r1.b and st4["outer_iterations"] == st1["outer_iterations"] >= 1


def test_distributed_oracle_failing_rank_ends_every_rank(prob2k, monkeypatch):
    """SVM355_DECOMP_FAIL_RANK / _OUTER: rank 2 fails at outer iteration 3 while its peers wait in the
    candidate all-gather; every rank leaves with the failing rank's error (no hang)."""
    from svm355._native import NativeError

    K, y = prob2k
    monkeypatch.setenv("SVM355_DECOMP_FAIL_RANK", "2")
    monkeypatch.setenv("SVM355_DECOMP_FAIL_OUTER", "3")
    with pytest.raises(NativeError, match="rank 2: .*injected failure of rank 2 at outer iteration 3"):
        C.decomp_train_gram_dist(K, y, SVMParams(n_threads=1), world=4, comm_timeout_s=30)


@pytest.mark.parametrize("env", [{"SVM355_DECOMP_NEWTON": "1"},
                                 {"SVM355_DECOMP_NEWTON": "1", "SVM355_DECOMP_NEWTON_EVERY": "3",
                                  "SVM355_DECOMP_NEWTON_FRAC": "0"},
                                 {"SVM355_DECOMP_NEWTON": "1", "SVM355_DECOMP_NEWTON_EVERY": "10",
                                  "SVM355_DECOMP_NEWTON_REPEAT": "5", "SVM355_DECOMP_NEWTON_MAX": "30"}])
def test_newton_polish_keeps_the_stop_test_and_the_svs(prob2k, monkeypatch, env):
    """The Newton polish of the working set's free variables (decomp_newton.h): the solve still meets the
    reference's stop test on all points with the pairwise solve's support vectors, and it takes fewer
    pair updates than the polish-free solve when it fires."""
    K, y = prob2k
    p = SVMParams(n_threads=4)
    a0, r0, st0, _ = C.decomp_train_gram(K, y, p)  # the default: no polish
    assert st0["newton_steps"] == 0
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    a, r, st, _ = C.decomp_train_gram(K, y, p)
    assert r.stop_reason == "converged" and _gap(K, y, a, p) <= 2 * p.tau + 1e-9
    np.testing.assert_array_equal(np.flatnonzero(a > p.sv_tol), np.flatnonzero(a0 > p.sv_tol))
    assert abs(r.b - r0.b) <= 10 * p.tau and abs(float(a @ y)) < 1e-9 * max(1.0, a.sum())
    assert np.all((a >= -1e-9) & (a <= p.C + 1e-9))  # the pairwise clip arithmetic rounds
    if env.get("SVM355_DECOMP_NEWTON_FRAC") == "0":  # a step at the start of every inner solve
        assert st["newton_steps"] >= 1
    if st["newton_steps"]:
        assert st["inner_iterations"] < st0["inner_iterations"]


def test_newton_step_solves_the_free_subproblem():
    """One step on a working set whose free points stay free (a well-separated RBF set: K close to I, so
    the free optimum alpha = 1 - mean(y) y is inside the box): afterwards every free point has the same f
    (the QP on F solved, to rounding), f is the kernel's f of the new alpha, and sum y alpha is unchanged."""
    from svm355._native import newton_step_probe

    rng = np.random.default_rng(3)
    m = 40
    X = rng.normal(size=(m, 5)) * 3.0
    sq = (X * X).sum(1)
    Kw = np.exp(-0.5 * np.maximum(sq[:, None] + sq[None, :] - 2 * X @ X.T, 0.0))
    np.fill_diagonal(Kw, 1.0)
    y = np.where(np.arange(m) % 3 == 0, 1, -1).astype(np.int32)
    a = rng.uniform(0.8, 1.2, size=m)
    a[y == 1] *= a[y == -1].sum() / a[y == 1].sum()  # sum y a = 0
    f = Kw @ (a * y) - y
    a2, f2, code = newton_step_probe(Kw, y, a, f, C=10.0)
    assert code == 1 and np.all((a2 > 0) & (a2 < 10.0))
    np.testing.assert_allclose(f2, Kw @ (a2 * y) - y, rtol=0, atol=1e-12)
    assert np.ptp(f2) < 1e-12
    assert abs(float(a2 @ y)) < 1e-12 * a2.sum()
    # cut at a bound: a box so small the step must stop at the first bound it meets
    a3, f3, code3 = newton_step_probe(Kw, y, a * 0.1, Kw @ (0.1 * a * y) - y, C=0.15)
    assert code3 == 2 and np.sum((a3 == 0.0) | (a3 == 0.15)) >= 1
    np.testing.assert_allclose(f3, Kw @ (a3 * y) - y, rtol=0, atol=1e-12)
