"""Degenerate inputs on the GPU trainers (the default decomposition solver and the pairwise SMO): a single
class, the smallest problems, constant and duplicate columns / rows, a single feature.  Each must end with
a reported stop reason (never a fault or a hang) and, where the problem is well-posed, the stop test."""
import numpy as np
import pytest

from svm355 import SVC

pytestmark = pytest.mark.gpu


def _gap(X, y, a, m):
    Xs = m.scaler_.transform(X) if m.scaler_ is not None else X
    sq = np.einsum("ij,ij->i", Xs, Xs)
    K = np.exp(-m.params.gamma * np.maximum(sq[:, None] + sq[None, :] - 2.0 * Xs @ Xs.T, 0.0))
    np.fill_diagonal(K, 1.0)
    yf = y.astype(np.float64)
    f = K @ (a * yf) - yf
    C, eps = m.params.C, m.params.eps
    hi = ((yf == 1) & (a < C - eps)) | ((yf == -1) & (a > eps))
    lo = ((yf == 1) & (a > eps)) | ((yf == -1) & (a < C - eps))
    return f[lo].max() - f[hi].min()


@pytest.mark.parametrize("solver", ["decomp", "smo"])
def test_single_class_reports_no_candidate(solver):
    rng = np.random.default_rng(1)
    X = rng.integers(0, 256, size=(300, 20)).astype(np.uint8)
    y = -np.ones(300, dtype=np.int32)
    m = SVC(device="cuda:0", solver=solver).fit(X, y)
    assert m.stop_reason_ == "no_candidate"
    assert np.all(m.alpha_ == 0.0)


@pytest.mark.parametrize("solver", ["decomp", "smo"])
@pytest.mark.parametrize("n", [2, 3, 17])
def test_smallest_problems(solver, n):
    rng = np.random.default_rng(n)
    X = rng.integers(0, 256, size=(n, 5)).astype(np.uint8)
    y = np.where(np.arange(n) % 2 == 0, 1, -1).astype(np.int32)
    m = SVC(device="cuda:0", solver=solver).fit(X, y)
    assert m.stop_reason_ == "converged"
    assert _gap(X.astype(np.float64), y, m.alpha_, m) <= 2 * m.params.tau + 1e-9


@pytest.mark.parametrize("solver", ["decomp", "smo"])
def test_constant_and_duplicate_columns_and_rows(solver):
    rng = np.random.default_rng(7)
    X = rng.integers(0, 256, size=(1500, 40)).astype(np.uint8)
    X[:, 3] = 17            # constant column (range 0: scaled to 0)
    X[:, 9] = X[:, 8]       # duplicate column
    X[100:200] = X[0:100]   # duplicate rows
    y = np.where(X[:, 0].astype(int) + X[:, 1] > 255, 1, -1).astype(np.int32)
    y[100:200] = y[0:100]
    m = SVC(device="cuda:0", solver=solver).fit(X, y)
    assert m.stop_reason_ == "converged"
    assert _gap(X.astype(np.float64), y, m.alpha_, m) <= 2 * m.params.tau + 1e-9


@pytest.mark.parametrize("solver", ["decomp", "smo"])
def test_single_feature_real_valued(solver):
    rng = np.random.default_rng(3)
    X = rng.standard_normal((800, 1))
    y = np.where(X[:, 0] + 0.3 * rng.standard_normal(800) > 0, 1, -1).astype(np.int32)
    m = SVC(device="cuda:0", solver=solver, gamma=1.0, C=1.0).fit(X, y)
    assert m.stop_reason_ == "converged"
    assert _gap(X, y, m.alpha_, m) <= 2 * m.params.tau + 1e-8


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_cascade_with_tiny_single_class_partitions(topology):
    """8 loopback ranks on 24 points sorted by label: every partition holds one class (no local solve
    finds a violating pair, no rank has a support vector): the cascade ends cleanly with an empty model."""
    from svm355.parallel.cascade import CascadeSVM

    rng = np.random.default_rng(11)
    X = rng.integers(0, 256, size=(24, 6)).astype(np.uint8)
    y = np.where(np.arange(24) < 12, 1, -1).astype(np.int32)  # ranks 0-3 all +1, ranks 4-7 all -1
    c = CascadeSVM(topology=topology).fit(X, y, world=8, device="cuda:0", transport="loopback")
    assert c.result.converged and len(c.result.ids) == 0 and c.result.b == 0.0


def test_distributed_decomposition_with_fewer_points_than_blocks():
    """8 rehearsal ranks on 40 points (the 8-block grain leaves ranks with one small block each)."""
    from svm355.parallel.decomp import DistributedDecompSVC

    rng = np.random.default_rng(12)
    X = rng.integers(0, 256, size=(40, 6)).astype(np.uint8)
    y = np.where(rng.random(40) < 0.5, 1, -1).astype(np.int32)
    y[0], y[1] = 1, -1
    one = SVC(device="cuda:0", solver="decomp").fit(X, y)
    m = DistributedDecompSVC(world=8, transport="loopback").fit(X, y)
    assert m.stop_reason_ == one.stop_reason_ == "converged"
    np.testing.assert_array_equal(m.alpha_, one.alpha_)


@pytest.mark.parametrize("bad", [np.nan, np.inf])
def test_non_finite_rows_are_rejected_on_the_gpu(bad):
    """FP64 rows with a NaN or an infinity: the device column bounds propagate NaN (fmin / fmax alone
    would drop it), and the fit raises instead of returning an empty model."""
    from svm355 import OneVsRestSVC

    rng = np.random.default_rng(5)
    X = rng.random((3000, 12))
    X[1234, 7] = bad
    y = np.where(rng.random(3000) < 0.5, 1, -1).astype(np.int32)
    for solver in ("decomp", "smo"):
        with pytest.raises(ValueError, match="NaN or infinite"):
            SVC(device="cuda:0", solver=solver).fit(X, y)
    with pytest.raises(ValueError, match="NaN or infinite"):
        OneVsRestSVC(device="cuda:0").fit(X, rng.integers(0, 3, size=3000))
    with pytest.raises(ValueError, match="NaN or infinite"):
        OneVsRestSVC(device="cuda:0", solver="batched").fit(X, rng.integers(0, 3, size=3000))


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_cascade_with_more_ranks_than_rows(topology):
    """8 loopback ranks on 5 rows: three partitions are empty (no upload, no min/max, no solve)."""
    from svm355.parallel.cascade import CascadeSVM

    rng = np.random.default_rng(13)
    X = rng.integers(0, 256, size=(5, 6)).astype(np.uint8)
    y = np.array([1, -1, 1, -1, 1], dtype=np.int32)
    c = CascadeSVM(topology=topology).fit(X, y, world=8, device="cuda:0", transport="loopback")
    assert c.result.converged


def test_distributed_decomposition_with_more_ranks_than_rows():
    from svm355.parallel.decomp import DistributedDecompSVC

    rng = np.random.default_rng(14)
    X = rng.integers(0, 256, size=(5, 6)).astype(np.uint8)
    y = np.array([1, -1, 1, -1, 1], dtype=np.int32)
    one = SVC(device="cuda:0", solver="decomp").fit(X, y)
    m = DistributedDecompSVC(world=8, transport="loopback").fit(X, y)
    assert m.stop_reason_ == one.stop_reason_ == "converged"
    np.testing.assert_array_equal(m.alpha_, one.alpha_)


@pytest.mark.parametrize("d", [1, 3, 17, 129, 1023, 3000])
@pytest.mark.parametrize("kind", ["u8", "f64"])
def test_feature_counts_from_1_to_3000(d, kind):
    """Odd and large feature counts (row strides padded to 16 doubles, k-steps of 32 / 128 int8 columns,
    the exact plan's step cap): the default GPU solver ends on the stop test, with the pairwise solver's
    support vectors."""
    rng = np.random.default_rng(d)
    n = 1500
    if kind == "u8":
        X = rng.integers(0, 256, size=(n, d)).astype(np.uint8)
        Xf = X.astype(np.float64)
    else:
        Xf = X = rng.standard_normal((n, d))
    w = rng.standard_normal(d)
    y = np.where(Xf @ w > np.median(Xf @ w), 1, -1).astype(np.int32)
    gamma = 1.0 / d  # the rows are min-max scaled to [0, 1] either way
    m = SVC(device="cuda:0", gamma=gamma).fit(X, y)
    p = SVC(device="cuda:0", gamma=gamma, solver="smo").fit(X, y)
    assert m.stop_reason_ == "converged" and p.stop_reason_ in ("converged", "max_iter")
    assert _gap(Xf, y, m.alpha_, m) <= 2 * m.params.tau + 1e-8
    if p.stop_reason_ == "converged":
        assert abs(len(m.support_) - len(p.support_)) <= max(2, len(p.support_) // 100)


@pytest.mark.parametrize("n", [2047, 2049, 16383, 16385, 65535, 65537])
def test_pairwise_solver_shape_boundaries(n):
    """The pairwise solver changes shape with n (one workgroup up to 2,048 points, 256- then 512-thread
    XCD-local teams up to 64k, the device-wide solver above): on both sides of each boundary it reaches the
    stop test with the decomposition solver's support vectors and b within 10 tau."""
    from svm355.utils.data import synthetic_mnist

    tr = synthetic_mnist(n, seed=n % 97).compact()
    p = SVC(device="cuda:0", solver="smo").fit(tr.X, tr.y)
    m = SVC(device="cuda:0").fit(tr.X, tr.y)
    assert p.stop_reason_ == m.stop_reason_ == "converged"
    np.testing.assert_array_equal(p.support_, m.support_)
    assert abs(p.b_ - m.b_) <= 10 * p.params.tau


def test_decomposition_beyond_2097152_rows():
    """Past 2,097,152 rows the selection keeps 512 blocks (their extreme pairs fill one working set) of more
    than 4,096 points each (ws_select_wide_kernel); the solve ends on the stop test, recomputed here from
    the exact-integer kernel values over all rows (two overlapping 8-dimensional pixel clusters)."""
    import torch

    from svm355.ops import device as D

    DEV = torch.device("cuda:0")
    n, d = 2_200_000, 8
    rng = np.random.default_rng(3)
    y = np.where(rng.random(n) < 0.5, 1, -1).astype(np.int32)
    X = np.clip(np.rint(np.where(y[:, None] > 0, 156.0, 100.0) + 25.0 * rng.standard_normal((n, d))), 0, 255)
    X = X.astype(np.uint8)
    m = SVC(device="cuda:0", solver="decomp", gamma=1.0 / d).fit(X, y)
    assert m.stop_reason_ == "converged" and m.timings_["solver"] == "decomp"
    assert m.support_.size > 100
    Xu = D.upload_u8(X, DEV)
    mmd = torch.empty(2 * d, dtype=torch.float64, device=DEV)
    D.minmax_u8(Xu, out=mmd)
    mm = mmd.cpu().numpy()
    f = -y.astype(np.float64)
    sv = np.flatnonzero(m.alpha_ > 0).astype(np.int32)  # every nonzero alpha, not only those above sv_tol
    coef = m.alpha_[sv] * y[sv]
    for k in range(0, sv.size, 1024):
        f += D.decomp_gemv_u8(Xu, mm[:d].copy(), mm[d:].copy(), 1.0 / d, sv[k:k + 1024], coef[k:k + 1024])
    a, p = m.alpha_, m.params
    hi = ((y == 1) & (a < p.C - p.eps)) | ((y == -1) & (a > p.eps))
    lo = ((y == 1) & (a > p.eps)) | ((y == -1) & (a < p.C - p.eps))
    assert f[lo].max() - f[hi].min() <= 2 * p.tau + 1e-9
