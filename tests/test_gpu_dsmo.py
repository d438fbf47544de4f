"""Distributed SMO (csrc/hip/dsmo.hip) on the one-GPU box: P teams in one launch stand in for P GPUs
(the rehearsal form: same kernel, same uncached receive arrays and system-scope exchange, the
records of every team written into every team's array).  The trajectory must be the single-GPU
resident solve's bit for bit: the whole (i_high, i_low) trace, every alpha and b."""
import numpy as np
import pytest
import torch

from svm355 import SVC, SVMParams
from svm355.parallel.dsmo import DistributedSVC, DsmoGroup
from svm355.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def D():
    from svm355.ops import device

    return device


def _single(D, tr, trace_cap):
    dev = torch.device("cuda:0")
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, tr.d)
    K, path = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    assert path == "int8-exact"
    yd = torch.from_numpy(tr.y).to(dev)
    a = torch.zeros(tr.n, dtype=torch.float64, device=dev)
    r, trc = D.smo(K, yd, a, SVMParams(), n=tr.n, trace_cap=trace_cap)
    del K
    return r, trc, a.cpu().numpy()


@pytest.mark.parametrize("n,world", [(3000, 1), (3000, 2), (6000, 3), (6000, 8), (20000, 4)])
def test_rehearsal_trajectory_equals_single_gpu(D, n, world):
    tr = synthetic_mnist(n, seed=31).compact()
    r1, t1, a1 = _single(D, tr, 200000)
    g = DsmoGroup(world, rehearsal=True)
    try:
        out = g.fit(tr.X, tr.y, SVMParams(), trace_cap=200000)
    finally:
        g.close()
    assert out["stop_reason"] == "converged"
    assert out["iterations"] == r1.iterations and out["b"] == r1.b
    np.testing.assert_array_equal(out["trace"], t1)
    np.testing.assert_array_equal(out["alpha"], a1)
    assert out["shape"]["workgroups_per_team"] >= 1


def test_rehearsal_at_the_headline_shape(D):
    """60k MNIST-shaped rows over 8 teams: the bench's solve (12,793 iterations), same b and SVs."""
    tr = synthetic_mnist(60000, seed=2024).compact()
    m1 = SVC(device="cuda:0", solver="smo").fit(tr.X, tr.y)
    g = DsmoGroup(8, rehearsal=True)
    try:
        m = DistributedSVC(8, rehearsal=True, group=g).fit(tr.X, tr.y)
        m2 = DistributedSVC(8, rehearsal=True, group=g).fit(tr.X, tr.y)  # buffers reused, epochs advance
    finally:
        g.close()
    assert m.n_iter_ == m1.n_iter_ == 12793 and m.b_ == m1.b_
    np.testing.assert_array_equal(m.support_, m1.support_)
    np.testing.assert_array_equal(m.alpha_, m1.alpha_)
    assert m2.b_ == m.b_ and m2.n_iter_ == m.n_iter_
    te = synthetic_mnist(2000, seed=2024, offset=60000).compact()
    assert m.score(te.X, te.y) == m1.score(te.X, te.y)


def test_non_pixel_data_are_refused():
    tr = synthetic_mnist(1000, seed=3)
    X = tr.X.copy()
    X[:, 5] += 0.5  # non-integer column: no exact-integer plan (the caller takes the cascade)
    g = DsmoGroup(2, rehearsal=True)
    try:
        with pytest.raises(ValueError, match="integer pixel rows"):
            g.fit(X, tr.y)
    finally:
        g.close()
