"""The decomposition solver's device kernels against host references.

* The f-update GEMV (``igram_tri_kernel`` GEMV mode + ``ws_fsum_count_kernel``) alone, against numpy
  ``K_exact[:, cols] @ coef`` (1e-13 relative) and bit for bit against the CPU emulation of its
  summation order (``svm_decomp_gemv_ref``): device-side counts of 1 / 63 / 64 / 65 / 1024 columns, both
  grid forms (fewer and more than 256 row tiles: n = 20k and 60k) and a distributed slice (row offset).
* The whole solve against its CPU oracle (``svm_decomp_train_gram``, csrc/core/decomp_cpu.cpp) given
  the device's own kernel values: every outer iteration's working set, moved columns, coefficients,
  inner iterations, bounds, alpha and f, bit for bit, at n = 2k / 6k and q = 64 / 512 / 1024, cold and
  warm started."""
import numpy as np
import pytest
import torch

from svm355 import SVC, SVMParams
from svm355 import _native as N
from svm355.ops import cpu as C
from svm355.ops import device as D
from svm355.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _dev_rows(tr):
    Xu = D.upload_u8(tr.X, DEV)
    mmd = torch.empty(2 * tr.d, dtype=torch.float64, device=DEV)
    mn, mx = D.minmax_u8(Xu, out=mmd)
    mm = mmd.cpu().numpy()
    return Xu, mm[: tr.d].copy(), mm[tr.d:].copy()


def _exact_gram_host(Xu, mn, mx, n, cols=None):
    K = D.rbf_gram_u8(Xu, 0.00125, mn, mx)
    assert K is not None
    if cols is not None:
        out = K[:n][:, torch.from_numpy(np.asarray(cols, dtype=np.int64)).to(DEV)].cpu().numpy()
    else:
        out = K[:n, :n].cpu().numpy()
    del K
    D.release_gram_buffers()
    torch.cuda.empty_cache()
    return np.ascontiguousarray(out)


@pytest.mark.parametrize("via", ["gemv", "cache"])
@pytest.mark.parametrize("n", [20000, 60000])
def test_gemv_against_numpy_and_its_summation_order(n, via, monkeypatch):
    """via="cache": the column-cache form of the update (every column stored -- the narrow store up to
    64 columns, the tiled one beyond -- then read back in the GEMV order) gives the same bits."""
    monkeypatch.setenv("SVM355_GEMV_VIA_CACHE", "1" if via == "cache" else "0")
    tr = synthetic_mnist(n, seed=31).compact()
    Xu, mn, mx = _dev_rows(tr)
    rng = np.random.default_rng(n)
    allc = np.sort(rng.choice(n, size=1024, replace=False)).astype(np.int32)
    Ksub = _exact_gram_host(Xu, mn, mx, n, allc)  # K(:, allc), the Gram's own values
    slices = [(0, n), (7501, 5000)] if n == 20000 else [(0, n)]
    for m in (1, 63, 64, 65, 1024):
        pick = np.sort(rng.choice(1024, size=m, replace=False))
        cols, coef = allc[pick], rng.uniform(-10.0, 10.0, size=m)
        for lo, nloc in slices:
            out = D.decomp_gemv_u8(Xu, mn, mx, 0.00125, cols, coef, lo, nloc)
            assert out is not None
            rows = np.ascontiguousarray(Ksub[lo:lo + nloc][:, pick])
            ref = np.zeros(nloc)
            idx = np.arange(m, dtype=np.int32)  # held: the native call reads it
            N.check(N.core().svm_decomp_gemv_ref(N.ptr(rows), rows.shape[1], nloc, N.ptr(idx), N.ptr(coef), m,
                                                 N.ptr(ref)), "svm_decomp_gemv_ref")
            np.testing.assert_array_equal(out, ref, err_msg=f"n={n} m={m} lo={lo}: summation order")
            exact = rows @ coef
            scale = np.abs(rows) @ np.abs(coef)
            assert np.all(np.abs(out - exact) <= 1e-13 * scale + 1e-300), f"n={n} m={m} lo={lo}"


def _compare(dt, ot):
    dr, orr = dt.records(), ot.records()
    assert len(dr) == len(orr) and len(dr) > 0
    for o, (a, b) in enumerate(zip(dr, orr)):
        assert a["m"] == b["m"], o
        np.testing.assert_array_equal(a["W"], b["W"], err_msg=f"outer {o}: working set")
        assert a["inner"] == b["inner"], o
        np.testing.assert_array_equal(a["bounds"], b["bounds"], err_msg=f"outer {o}: bounds")
        np.testing.assert_array_equal(a["cols"], b["cols"], err_msg=f"outer {o}: moved columns")
        np.testing.assert_array_equal(a["coef"], b["coef"], err_msg=f"outer {o}: coefficients")
        np.testing.assert_array_equal(a["alpha"], b["alpha"], err_msg=f"outer {o}: alpha")
        np.testing.assert_array_equal(a["f"], b["f"], err_msg=f"outer {o}: f")


@pytest.mark.parametrize("n,q,wss", [(2000, 1024, 3), (2000, 64, 3), (6000, 512, 3), (6000, 1024, 3),
                                     (2000, 1024, 4), (6000, 1024, 4)])
def test_device_trajectory_equals_the_cpu_oracle(n, q, wss, monkeypatch):
    # wss 4: the second pair's j by the second-order gain of row i2 (SVM355_DECOMP_WSS=4, oracle inner_wss 4)
    monkeypatch.setenv("SVM355_DECOMP_WSS", str(wss))
    tr = synthetic_mnist(n, seed=41 + q).compact()
    Xu, mn, mx = _dev_rows(tr)
    K = _exact_gram_host(Xu, mn, mx, n)
    p = SVMParams()
    yd = torch.from_numpy(tr.y).to(DEV)
    alpha = torch.empty(n, dtype=torch.float64, device=DEV)
    dt = N.DecompTrace(400, n)
    res, tm = D.train_decomp(Xu, yd, alpha, p, mn, mx, working_set=q, trace=dt)
    a_o, r_o, st_o, ot = C.decomp_train_gram(K, tr.y, SVMParams(n_threads=8), q=q, inner_wss=wss, trace_cap=400,
                                             snapshots=True)
    _compare(dt, ot)
    assert res.stop_reason == r_o.stop_reason == "converged"
    assert res.iterations == r_o.iterations and res.b == r_o.b
    np.testing.assert_array_equal(alpha.cpu().numpy(), a_o)
    assert tm["outer_iterations"] == st_o["outer_iterations"] and tm["working_set"] == st_o["working_set"]


def test_warm_start_equals_the_oracle_and_meets_the_stop_test():
    """A cascade-shaped warm start: the solution of the first half (feasible for the whole problem,
    zero elsewhere) starts the solve on all rows; the device's warm f and trajectory are the oracle's,
    and the KKT gap recomputed from the exact Gram is within 2 tau."""
    n = 6000
    tr = synthetic_mnist(n, seed=55).compact()
    Xu, mn, mx = _dev_rows(tr)
    K = _exact_gram_host(Xu, mn, mx, n)
    p = SVMParams()
    half = tr.subset(0, n // 2)
    a_half = SVC(device="cuda:0", solver="decomp").fit(half.X, half.y).alpha_
    a0 = np.concatenate([a_half, np.zeros(n - n // 2)])
    yd = torch.from_numpy(tr.y).to(DEV)
    alpha = torch.from_numpy(a0.copy()).to(DEV)
    dt = N.DecompTrace(400, n)
    res, tm = D.train_decomp(Xu, yd, alpha, p, mn, mx, warm=True, trace=dt)
    a_o, r_o, st_o, ot = C.decomp_train_gram(K, tr.y, SVMParams(n_threads=8), alpha=a0, trace_cap=400, snapshots=True)
    _compare(dt, ot)
    a = alpha.cpu().numpy()
    np.testing.assert_array_equal(a, a_o)
    assert res.stop_reason == "converged" and res.b == r_o.b and tm["warm_start"]
    y = tr.y.astype(np.float64)
    f = K @ (a * y) - y
    hi = ((y == 1) & (a < p.C - p.eps)) | ((y == -1) & (a > p.eps))
    lo = ((y == 1) & (a > p.eps)) | ((y == -1) & (a < p.C - p.eps))
    assert f[lo].max() - f[hi].min() <= 2 * p.tau + 1e-9
    cold = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    np.testing.assert_array_equal(np.flatnonzero(a > p.sv_tol), cold.support_)
    warm = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y, alpha0=a0)  # the estimator's warm start
    np.testing.assert_array_equal(warm.alpha_, a)


@pytest.mark.parametrize("slots,evict", [(None, None), ("300", None), ("8", None), ("300", "0")])
def test_column_cache_trajectory_equals_the_oracle(monkeypatch, slots, evict):
    """The f update served from the column cache (forced on at 6k) keeps the oracle's trajectory bit for
    bit, cold and warm: with every column cached; with 300 slots (the cache fills, then the CLOCK sweep
    evicts slots the update does not read); with 8 (fewer slots than a sweep's window: the hand wraps,
    most misses take scratch slots); and with 300 fill-only slots (SVM355_DECOMP_CCACHE_EVICT=0)."""
    monkeypatch.setenv("SVM355_DECOMP_CCACHE", "1")
    if slots:
        monkeypatch.setenv("SVM355_DECOMP_CCACHE_SLOTS", slots)
    if evict:
        monkeypatch.setenv("SVM355_DECOMP_CCACHE_EVICT", evict)
    n = 6000
    tr = synthetic_mnist(n, seed=61).compact()
    Xu, mn, mx = _dev_rows(tr)
    K = _exact_gram_host(Xu, mn, mx, n)
    yd = torch.from_numpy(tr.y).to(DEV)
    half = tr.subset(0, n // 2)
    a_half = SVC(device="cuda:0", solver="decomp").fit(half.X, half.y).alpha_
    for warm in (False, True):
        a0 = np.concatenate([a_half, np.zeros(n - n // 2)]) if warm else np.zeros(n)
        alpha = torch.from_numpy(a0.copy()).to(DEV)
        dt = N.DecompTrace(400, n)
        res, tm = D.train_decomp(Xu, yd, alpha, SVMParams(), mn, mx, warm=warm, trace=dt)
        a_o, r_o, st_o, ot = C.decomp_train_gram(K, tr.y, SVMParams(n_threads=8), alpha=a0 if warm else None,
                                                 trace_cap=400, snapshots=True)
        _compare(dt, ot)
        a = alpha.cpu().numpy()
        np.testing.assert_array_equal(a, a_o)
        assert res.stop_reason == r_o.stop_reason == "converged" and res.b == r_o.b


@pytest.mark.parametrize("n,slots", [(60000, None), (250000, None), (250000, "1500")])
def test_column_cache_is_bit_identical_at_large_n(monkeypatch, n, slots):
    """The cache (SVM355_DECOMP_CCACHE=1; the default from ~200k rows) against the GEMV path
    (SVM355_DECOMP_CCACHE=0): the same alpha, b and iteration counts -- also with 1,500 slots for the
    ~3,000 distinct columns of the 250k solve (eviction in most late updates)."""
    if slots:
        monkeypatch.setenv("SVM355_DECOMP_CCACHE_SLOTS", slots)
    tr = synthetic_mnist(n, seed=2024).compact()
    Xu, mn, mx = _dev_rows(tr)
    yd = torch.from_numpy(tr.y).to(DEV)
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("SVM355_DECOMP_CCACHE", flag)
        alpha = torch.empty(n, dtype=torch.float64, device=DEV)
        res, tm = D.train_decomp(Xu, yd, alpha, SVMParams(), mn, mx)
        out[flag] = (alpha.cpu().numpy(), res.b, res.iterations, tm["outer_iterations"], res.stop_reason)
    np.testing.assert_array_equal(out["0"][0], out["1"][0])
    assert out["0"][1:] == out["1"][1:] and out["1"][4] == "converged"


@pytest.mark.parametrize("d,kww", [(784, "sym"), (1800, None)])
def test_kww_paths_equal_the_oracle(monkeypatch, d, kww):
    """K(W, W) from the triangular Gram launch (SVM355_DECOMP_KWW=sym; and, automatically, for rows
    wider than the narrow store's 1,536 int8 columns) instead of the narrow column store: the same
    trajectory as the CPU oracle, bit for bit."""
    if kww:
        monkeypatch.setenv("SVM355_DECOMP_KWW", kww)
    n = 3000
    rng = np.random.default_rng(d)
    X = rng.integers(0, 256, size=(n, d)).astype(np.uint8)
    X[:, : d // 3] = np.minimum(X[:, : d // 3], 12)  # an extra column group (12 does not divide 255)
    y = np.where(X[:, :64].astype(np.int64).sum(1) > np.median(X[:, :64].astype(np.int64).sum(1)), 1, -1).astype(np.int32)
    Xu = D.upload_u8(X, DEV)
    mmd = torch.empty(2 * d, dtype=torch.float64, device=DEV)
    D.minmax_u8(Xu, out=mmd)
    mm = mmd.cpu().numpy()
    mn, mx = mm[:d].copy(), mm[d:].copy()
    K = _exact_gram_host(Xu, mn, mx, n)
    yd = torch.from_numpy(y).to(DEV)
    alpha = torch.empty(n, dtype=torch.float64, device=DEV)
    dt = N.DecompTrace(400, n)
    res, tm = D.train_decomp(Xu, yd, alpha, SVMParams(), mn, mx, trace=dt)
    assert tm["gram_path"] == "int8-exact"
    a_o, r_o, st_o, ot = C.decomp_train_gram(K, y, SVMParams(n_threads=8), trace_cap=400, snapshots=True)
    _compare(dt, ot)
    np.testing.assert_array_equal(alpha.cpu().numpy(), a_o)
    assert res.b == r_o.b and res.stop_reason == r_o.stop_reason


@pytest.mark.parametrize("n,q", [(2000, 1024), (6000, 64), (6000, 1024)])
def test_streamed_selection_equals_the_cpu_oracle(n, q, monkeypatch):
    """ws_select_wide_kernel, the selection past 2,097,152 rows (blocks of more than 4,096 points), forced
    at any n by SVM355_DECOMP_WIDE_SELECT=1: its T rounds of 'the best point after the previous pick'
    (T = 16 / 1 / 8 here) give the oracle's picks, so the whole trajectory stays the oracle's bit for bit."""
    monkeypatch.setenv("SVM355_DECOMP_WIDE_SELECT", "1")
    tr = synthetic_mnist(n, seed=77 + q).compact()
    Xu, mn, mx = _dev_rows(tr)
    K = _exact_gram_host(Xu, mn, mx, n)
    yd = torch.from_numpy(tr.y).to(DEV)
    alpha = torch.empty(n, dtype=torch.float64, device=DEV)
    dt = N.DecompTrace(400, n)
    res, tm = D.train_decomp(Xu, yd, alpha, SVMParams(), mn, mx, working_set=q, trace=dt)
    a_o, r_o, st_o, ot = C.decomp_train_gram(K, tr.y, SVMParams(n_threads=8), q=q, trace_cap=400, snapshots=True)
    _compare(dt, ot)
    assert res.stop_reason == r_o.stop_reason == "converged"
    assert res.iterations == r_o.iterations and res.b == r_o.b
    np.testing.assert_array_equal(alpha.cpu().numpy(), a_o)


AGGRESSIVE = {"SVM355_DECOMP_SHRINK": "1", "SVM355_DECOMP_SHRINK_START": "1", "SVM355_DECOMP_SHRINK_MARGIN": "0"}


@pytest.mark.parametrize("mode,cache,repack", [("aggressive", "0", None), ("aggressive", "0", "1.0"),
                                               ("aggressive", "1", "1.0"), ("period2", "1", None),
                                               ("aggressive", "1", "0")])
def test_shrinking_trajectory_equals_the_oracle(monkeypatch, mode, cache, repack):
    """Shrinking (decomp_shrink.h) on the device -- the shrink passes, the packed active rows (the GEMV /
    column store over them, their unit diagonal from packed positions, the column cache cleared at every
    repack; SVM355_DECOMP_REPACK=1.0 repacks after every drop, 0 never), the unshrink with f recomputed
    from alpha -- against the CPU oracle's trajectory bit for bit, cold and warm; f is compared on the
    active points (NaN elsewhere on both sides)."""
    for k, v in (AGGRESSIVE if mode == "aggressive" else {"SVM355_DECOMP_SHRINK": "2"}).items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("SVM355_DECOMP_CCACHE", cache)
    if repack is not None:
        monkeypatch.setenv("SVM355_DECOMP_REPACK", repack)
    n = 6000
    tr = synthetic_mnist(n, seed=61).compact()
    Xu, mn, mx = _dev_rows(tr)
    K = _exact_gram_host(Xu, mn, mx, n)
    yd = torch.from_numpy(tr.y).to(DEV)
    half = tr.subset(0, n // 2)
    a_half = SVC(device="cuda:0", solver="decomp").fit(half.X, half.y).alpha_
    for warm in (False, True):
        a0 = np.concatenate([a_half, np.zeros(n - n // 2)]) if warm else np.zeros(n)
        alpha = torch.from_numpy(a0.copy()).to(DEV)
        dt = N.DecompTrace(400, n)
        res, tm = D.train_decomp(Xu, yd, alpha, SVMParams(), mn, mx, warm=warm, trace=dt)
        a_o, r_o, st_o, ot = C.decomp_train_gram(K, tr.y, SVMParams(n_threads=8), alpha=a0 if warm else None,
                                                 trace_cap=400, snapshots=True)
        _compare(dt, ot)
        a = alpha.cpu().numpy()
        np.testing.assert_array_equal(a, a_o)
        assert res.stop_reason == r_o.stop_reason == "converged" and res.b == r_o.b
        assert tm["unshrinks"] == st_o["unshrinks"] and tm["shrink_passes"] == st_o["shrink_passes"]
        if mode == "aggressive":
            assert tm["unshrinks"] >= 1 and tm["min_active"] < n // 2
            if repack != "0":
                assert tm["repacks"] >= 1


def _kkt_gap_fp64(X, y, a, p):
    """b_low - b_high over ALL points from an independent FP64 RBF (torch, min-max scaled rows)."""
    Xs = torch.from_numpy(X.astype(np.float64)).to(DEV)
    mn, mx = Xs.min(0).values, Xs.max(0).values
    rng = torch.where(mx - mn < 1e-12, torch.ones_like(mx), mx - mn)
    Xs = (Xs - mn) / rng
    sq = (Xs * Xs).sum(1)
    ay = torch.from_numpy(a * y).to(DEV)
    f = torch.empty(len(y), dtype=torch.float64, device=DEV)
    for i0 in range(0, len(y), 4096):
        B = Xs[i0:i0 + 4096] @ Xs.T
        Kb = torch.exp(-p.gamma * torch.clamp(sq[i0:i0 + 4096, None] + sq[None, :] - 2.0 * B, min=0.0))
        f[i0:i0 + 4096] = Kb @ ay
    f = f.cpu().numpy() - y
    hi = ((y == 1) & (a < p.C - p.eps)) | ((y == -1) & (a > p.eps))
    lo = ((y == 1) & (a > p.eps)) | ((y == -1) & (a < p.C - p.eps))
    return f[lo].max() - f[hi].min()


@pytest.mark.parametrize("n", [60000])
def test_shrunk_solve_meets_the_stop_test_on_all_points(n):
    """The headline shape with shrinking=True against the default (off): the same support
    vectors, b within the stop tolerance, and the reference's stop test recomputed on all n points from
    an independent FP64 kernel (not the solver's int8-exact values, and not its f)."""
    tr = synthetic_mnist(n, seed=2024).compact()
    p = SVMParams()
    on = SVC(device="cuda:0", solver="decomp", shrinking=True).fit(tr.X, tr.y)
    off = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    np.testing.assert_array_equal(on.support_, off.support_)
    assert abs(on.b_ - off.b_) <= 10 * p.tau
    assert on.timings_["shrink_passes"] >= 1 and on.timings_["min_active"] < n
    assert off.timings_["shrink_passes"] == 0
    y = tr.y.astype(np.float64)
    assert _kkt_gap_fp64(tr.X, y, on.alpha_, p) <= 2 * p.tau + 1e-9


@pytest.mark.parametrize("env", [{"SVM355_DECOMP_NEWTON": "1", "SVM355_DECOMP_NEWTON_EVERY": "5", "SVM355_DECOMP_NEWTON_FRAC": "0"},
                                 {"SVM355_DECOMP_NEWTON": "1", "SVM355_DECOMP_NEWTON_EVERY": "20", "SVM355_DECOMP_NEWTON_REPEAT": "4",
                                  "SVM355_DECOMP_SHRINK": "1", "SVM355_DECOMP_SHRINK_START": "1"},
                                 {"SVM355_DECOMP_NEWTON": "1", "SVM355_DECOMP_NEWTON_EVERY": "10", "SVM355_DECOMP_CCACHE": "1",
                                  "SVM355_DECOMP_NEWTON_FRAC": "0", "SVM355_DECOMP_NEWTON_MAX": "150"}])
def test_newton_polish_trajectory_equals_the_oracle(monkeypatch, env):
    """The Newton polish of the working set's free variables (decomp_newton.h, newton_wg in the inner
    solve: a left-looking panel Cholesky of K_FF with two right-hand-side rows, the back substitution in
    one wave, the cut at the first bound) against the oracle's sequential reference, bit for bit: every
    working set, moved column, coefficient, alpha and f; forced often here (every 5-20 quiet chain
    iterations, from the first working set), with shrinking, with the column cache and a small |F| cap."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    fired = 0
    for n, seed in ((2000, 5), (6000, 61)):
        tr = synthetic_mnist(n, seed=seed).compact()
        Xu, mn, mx = _dev_rows(tr)
        K = _exact_gram_host(Xu, mn, mx, n)
        yd = torch.from_numpy(tr.y).to(DEV)
        alpha = torch.empty(n, dtype=torch.float64, device=DEV)
        dt = N.DecompTrace(400, n)
        res, tm = D.train_decomp(Xu, yd, alpha, SVMParams(), mn, mx, trace=dt)
        a_o, r_o, st_o, ot = C.decomp_train_gram(K, tr.y, SVMParams(n_threads=8), trace_cap=400, snapshots=True)
        _compare(dt, ot)
        np.testing.assert_array_equal(alpha.cpu().numpy(), a_o)
        assert res.stop_reason == r_o.stop_reason == "converged" and res.b == r_o.b
        assert tm["newton_steps"] == st_o["newton_steps"], (tm["newton_steps"], st_o["newton_steps"])
        fired += tm["newton_steps"]
    assert fired >= 1
