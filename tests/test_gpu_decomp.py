"""Working-set decomposition SMO (csrc/hip/decomp.hip, ``SVC(solver="decomp")``) against the
reference's pairwise solve (``solver="smo"``) on the same rows.  The two reach the same stop test on
all n points by different pair sequences, so the checks are the optimality conditions themselves
(recomputed on the host from the final alphas and an independent Gram), the support-vector set and
b within the stop tolerance -- not a bit-identical trajectory."""
import time

import numpy as np
import pytest
import torch

from svm355 import SVC, SVMParams
from svm355.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu


def _kkt_gap(D, tr, alpha, p: SVMParams):
    """b_low - b_high of the final alphas with f recomputed from the exact-integer Gram (float64)."""
    dev = torch.device("cuda:0")
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, tr.d)
    K, path = D.rbf_gram_sym(Xd, sqn, p.gamma, mn=mn, mx=mx)
    assert path == "int8-exact"
    K = K[: tr.n, : tr.n].cpu().numpy()
    y = tr.y.astype(np.float64)
    f = K @ (alpha * y) - y
    C, eps = p.C, p.eps
    hi = ((y == 1) & (alpha < C - eps)) | ((y == -1) & (alpha > eps))
    lo = ((y == 1) & (alpha > eps)) | ((y == -1) & (alpha < C - eps))
    return f[lo].max() - f[hi].min()


@pytest.mark.parametrize("n,q", [(2000, 1024), (6000, 512), (6000, 64)])
def test_decomp_meets_the_stop_test_with_the_pairwise_svs(n, q):
    from svm355.ops import device as D

    tr = synthetic_mnist(n, seed=77).compact()
    ref = SVC(device="cuda:0", solver="smo").fit(tr.X, tr.y)
    m = SVC(device="cuda:0", solver="decomp", working_set=q).fit(tr.X, tr.y)
    assert m.stop_reason_ == ref.stop_reason_ == "converged"
    assert m.timings_["solver"] == "decomp" and m.timings_["outer_iterations"] >= 1
    assert m.timings_["inner_iterations"] + 1 == m.n_iter_
    p = SVMParams()
    # the reference's stop test b_low <= b_high + 2 tau on all n points, with an independent f
    assert _kkt_gap(D, tr, m.alpha_, p) <= 2 * p.tau + 1e-9
    # each solve stops somewhere in its own band b_high <= b <= b_low (width <= 2 tau); the two bands
    # come from different approximate optima, so b agrees to a few tau, not bit for bit
    assert abs(m.b_ - ref.b_) <= 10 * p.tau
    np.testing.assert_array_equal(m.support_, ref.support_)
    assert np.all((m.alpha_ >= -1e-9) & (m.alpha_ <= p.C + 1e-9))  # the clip arithmetic rounds
    assert abs(float(np.dot(m.alpha_, tr.y))) < 1e-9 * max(1.0, m.alpha_.sum())
    te = synthetic_mnist(1000, seed=78).compact()
    agree = np.mean(m.predict(te.X) == ref.predict(te.X))
    assert agree >= 0.999


def test_decomp_at_the_headline_shape():
    """60k MNIST-shaped rows (the bench's problem): the same SV set as the pairwise solve and b
    within the stop tolerance, with far fewer device round trips (one per outer iteration)."""
    tr = synthetic_mnist(60000, seed=2024).compact()
    ref = SVC(device="cuda:0", solver="smo").fit(tr.X, tr.y)
    m = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    assert m.stop_reason_ == "converged"
    assert abs(m.b_ - ref.b_) <= 1e-4
    np.testing.assert_array_equal(m.support_, ref.support_)
    assert m.timings_["outer_iterations"] < 500


def test_decomp_fp64_rows_equal_the_byte_path():
    """FP64 host rows (the reference's format) are scaled on the device and quantised into the same
    integers as the uint8 rows: the same trajectory, alphas, b and predictions."""
    tr = synthetic_mnist(6000, seed=79).compact()
    a = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    b = SVC(device="cuda:0", solver="decomp").fit(tr.X.astype(np.float64), tr.y)
    assert b.timings_["rows"] == "fp64" and a.timings_["rows"] == "uint8"
    assert a.n_iter_ == b.n_iter_ and a.b_ == b.b_
    np.testing.assert_array_equal(a.alpha_, b.alpha_)
    te = synthetic_mnist(500, seed=80).compact()
    np.testing.assert_array_equal(a.predict(te.X), b.predict(te.X.astype(np.float64)))


def test_decomp_stop_reasons_of_the_device_loop():
    """The outer loop runs on a device-side control block (batches of launches, no host read per outer
    iteration): the iteration cap still stops it with the reference's reason and count, and every batch
    size gives the same model."""
    import os

    tr = synthetic_mnist(6000, seed=81).compact()
    m = SVC(device="cuda:0", solver="decomp", max_iter=300).fit(tr.X, tr.y)
    assert m.stop_reason_ == "max_iter" and m.n_iter_ == 301  # the reference counts from 1
    ref = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    old = os.environ.get("SVM355_DECOMP_BATCH")
    try:
        os.environ["SVM355_DECOMP_BATCH"] = "5"
        m5 = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    finally:
        if old is None:
            os.environ.pop("SVM355_DECOMP_BATCH", None)
        else:
            os.environ["SVM355_DECOMP_BATCH"] = old
    assert m5.n_iter_ == ref.n_iter_ and m5.b_ == ref.b_
    np.testing.assert_array_equal(m5.alpha_, ref.alpha_)
    assert m5.timings_["outer_iterations"] == ref.timings_["outer_iterations"]


def test_decomp_refuses_unscaled_rows():
    tr = synthetic_mnist(500, seed=3)
    with pytest.raises(ValueError, match="scale=True"):
        SVC(device="cuda:0", solver="decomp", scale=False).fit(tr.compact().X, tr.y)
    m = SVC(device="cuda:0", scale=False).fit(tr.compact().X, tr.y)  # auto: the pairwise solver then
    assert m.timings_.get("solver") != "decomp"


@pytest.mark.parametrize("n,d", [(3000, 50), (2500, 784)])
def test_decomp_on_real_valued_rows(n, d):
    """Rows with no exact-integer plan (real-valued data) are solved on the FP64 rows, every kernel
    value on FP64 MFMA (gram_mfma.hip): the KKT gap from numpy exp(-gamma d^2) is within 2 tau, and the
    support vectors are the pairwise FP64 solve's."""
    rng = np.random.default_rng(n + d)
    X = rng.random((n, d))
    w = rng.standard_normal(d)
    y = np.where(X @ w + 0.3 * rng.standard_normal(n) > np.median(X @ w), 1, -1).astype(np.int32)
    gamma, C = (0.05, 2.0) if d == 50 else (0.00125, 10.0)
    m = SVC(device="cuda:0", gamma=gamma, C=C).fit(X, y)
    assert m.timings_["solver"] == "decomp" and m.timings_["gram_path"] == "fp64"
    assert m.stop_reason_ == "converged"
    ref = SVC(device="cuda:0", gamma=gamma, C=C, solver="smo").fit(X, y)
    assert ref.timings_["gram_path"] == "fp64"
    Xs = (X - X.min(0)) / np.where(X.max(0) - X.min(0) < 1e-12, 1.0, X.max(0) - X.min(0))
    sq = np.einsum("ij,ij->i", Xs, Xs)
    K = np.exp(-gamma * np.maximum(sq[:, None] + sq[None, :] - 2.0 * Xs @ Xs.T, 0.0))
    np.fill_diagonal(K, 1.0)
    a, yf, p = m.alpha_, y.astype(np.float64), m.params
    f = K @ (a * yf) - yf
    hi = ((yf == 1) & (a < C - p.eps)) | ((yf == -1) & (a > p.eps))
    lo = ((yf == 1) & (a > p.eps)) | ((yf == -1) & (a < C - p.eps))
    assert f[lo].max() - f[hi].min() <= 2 * p.tau + 1e-8
    np.testing.assert_array_equal(m.support_, ref.support_)
    assert abs(m.b_ - ref.b_) <= 10 * p.tau


def test_decomp_f64_rows_forced_on_pixel_data(monkeypatch):
    """SVM355_DECOMP_F64=1 takes the FP64-MFMA path on pixel rows too: the kernel values agree with the
    exact-integer ones to a few ulps, so the model is the same to the stop tolerance."""
    tr = synthetic_mnist(4000, seed=83)
    a = SVC(device="cuda:0").fit(tr.X, tr.y)
    monkeypatch.setenv("SVM355_DECOMP_F64", "1")
    b = SVC(device="cuda:0").fit(tr.X, tr.y)
    assert a.timings_["gram_path"] == "int8-exact" and b.timings_["gram_path"] == "fp64"
    np.testing.assert_array_equal(a.support_, b.support_)
    assert abs(a.b_ - b.b_) <= 10 * a.params.tau
    assert np.mean(a.predict(tr.X) == b.predict(tr.X)) >= 0.999


def test_decomp_rejects_an_inner_stop_that_cannot_progress(monkeypatch):
    """At tau_frac >= 0.5 the working set's stop holds before any update: an error, not a zero model."""
    tr = synthetic_mnist(2000, seed=4).compact()
    monkeypatch.setenv("SVM355_DECOMP_TAU_FRAC", "0.5")
    with pytest.raises(Exception, match="TAU_FRAC"):
        SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    monkeypatch.setenv("SVM355_DECOMP_TAU_FRAC", "0.3")
    m = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    assert m.stop_reason_ == "converged" and len(m.support_) > 0


@pytest.mark.parametrize("n,world,ccache", [(6000, 2, None), (6000, 8, None), (20000, 4, None), (6000, 2, "1"),
                                             (20000, 4, "300")])
def test_distributed_rehearsal_equals_one_gpu(n, world, ccache, monkeypatch):
    """P ranks rehearsed on the one GPU (loopback transport, thread ranks): the global block partition
    makes every working set, alpha, b and iteration count the one-GPU decomposition solver's.  ccache:
    the column cache forced on (each rank caches its own rows' slice: row offsets in the store and the
    diagonal), "300": with 300 slots per rank (full caches, scratch slots)."""
    from svm355.parallel.decomp import DistributedDecompSVC
    from svm355.parallel.rccl import DeviceGroup

    if ccache:
        monkeypatch.setenv("SVM355_DECOMP_CCACHE", "1")
        if ccache != "1":
            monkeypatch.setenv("SVM355_DECOMP_CCACHE_SLOTS", ccache)

    tr = synthetic_mnist(n, seed=91).compact()
    one = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    g = DeviceGroup(world, "loopback")
    try:
        m = DistributedDecompSVC(world, group=g).fit(tr.X, tr.y)
    finally:
        g.close()
    assert m.stop_reason_ == "converged"
    assert m.n_iter_ == one.n_iter_ and m.b_ == one.b_
    np.testing.assert_array_equal(m.alpha_, one.alpha_)
    assert m.stats_["outer_iterations"] == one.timings_["outer_iterations"]
    te = synthetic_mnist(500, seed=92).compact()
    np.testing.assert_array_equal(m.predict(te.X), one.predict(te.X))


def _real_problem(n, d, seed):
    rng = np.random.default_rng(seed)
    X = rng.random((n, d))
    w = rng.standard_normal(d)
    y = np.where(X @ w + 0.3 * rng.standard_normal(n) > np.median(X @ w), 1, -1).astype(np.int32)
    return X, y


@pytest.mark.parametrize("world", [2, 4, 8])
def test_distributed_rehearsal_on_real_valued_rows_equals_one_gpu(world):
    """the distributed decomposition on FP64 real-valued rows (no exact-integer plan:
    every kernel value on FP64 MFMA, each rank's f update over its own rows) -- P thread ranks rehearsed on
    the one GPU give alpha, b and the iteration counts of the one-GPU FP64 decomposition bit for bit, and
    the reference's stop test holds against a numpy RBF (the reference's MPI programs partition double
    rows: mpi_svm_main2.cpp:316-402)."""
    from svm355.parallel.decomp import DistributedDecompSVC
    from svm355.parallel.rccl import DeviceGroup

    X, y = _real_problem(6000, 50, 7)
    gamma, C = 0.05, 2.0
    one = SVC(device="cuda:0", solver="decomp", gamma=gamma, C=C).fit(X, y)
    assert one.timings_["gram_path"] == "fp64"
    g = DeviceGroup(world, "loopback")
    try:
        m = DistributedDecompSVC(world, group=g, gamma=gamma, C=C).fit(X, y)
    finally:
        g.close()
    assert m.stop_reason_ == "converged"
    assert m.n_iter_ == one.n_iter_ and m.b_ == one.b_
    np.testing.assert_array_equal(m.alpha_, one.alpha_)
    Xs = (X - X.min(0)) / np.where(X.max(0) - X.min(0) < 1e-12, 1.0, X.max(0) - X.min(0))
    sq = np.einsum("ij,ij->i", Xs, Xs)
    K = np.exp(-gamma * np.maximum(sq[:, None] + sq[None, :] - 2.0 * Xs @ Xs.T, 0.0))
    np.fill_diagonal(K, 1.0)
    a, yf, p = m.alpha_, y.astype(np.float64), m.params
    f = K @ (a * yf) - yf
    hi = ((yf == 1) & (a < C - p.eps)) | ((yf == -1) & (a > p.eps))
    lo = ((yf == 1) & (a > p.eps)) | ((yf == -1) & (a < C - p.eps))
    assert f[lo].max() - f[hi].min() <= 2 * p.tau + 1e-8
    te, _ = _real_problem(500, 50, 8)
    np.testing.assert_array_equal(m.predict(te), one.predict(te))


@pytest.mark.parametrize("d,world", [(4096, 2), (4160, 2), (4160, 4)])
def test_distributed_rehearsal_at_the_int8_column_bound(d, world):
    """VERDICT r5 item 4 (the kq > 4,096 boundary): pixel rows with d columns of range 255 need d int8
    columns (padded to 64).  Up to 4,096 they take the exact-integer plan; past it no plan fits the int8
    kernels, and the distributed entry solves them as FP64 rows (every rank the same way: the plan is a
    function of the global min / max), as the one-GPU SVC does -- alpha, b and the iterations equal the
    one-GPU fit bit for bit at both sides of the bound."""
    from svm355.parallel.decomp import DistributedDecompSVC
    from svm355.parallel.rccl import DeviceGroup

    rng = np.random.default_rng(d)
    n = 1500
    X = rng.integers(0, 256, size=(n, d), dtype=np.uint8)
    X[0], X[1] = 0, 255  # every column's range is 255
    w = rng.standard_normal(d)
    sc = X.astype(np.float64) @ w
    y = np.where(sc > np.median(sc), 1, -1).astype(np.int32)
    one = SVC(device="cuda:0", solver="decomp").fit(X, y)
    assert one.timings_["gram_path"] == ("int8-exact" if d <= 4096 else "fp64"), one.timings_["gram_path"]
    g = DeviceGroup(world, "loopback")
    try:
        m = DistributedDecompSVC(world, group=g).fit(X, y)
    finally:
        g.close()
    assert m.stop_reason_ == "converged"
    assert m.n_iter_ == one.n_iter_ and m.b_ == one.b_
    np.testing.assert_array_equal(m.alpha_, one.alpha_)


def test_distributed_process_rank_world1_equals_one_gpu():
    """The per-process entry (torchrun form, RCCL communicator of one rank) on the one GPU."""
    from svm355.parallel.decomp import DistributedDecompSVC
    from svm355.parallel.rccl import RcclRank

    tr = synthetic_mnist(4000, seed=93).compact()
    one = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    rk = RcclRank(0, RcclRank.unique_id(), 1, 0)
    try:
        m = DistributedDecompSVC(rank=rk).fit(tr.X, tr.y)
    finally:
        rk.close()
    assert m.n_iter_ == one.n_iter_ and m.b_ == one.b_
    np.testing.assert_array_equal(m.alpha_, one.alpha_)


@pytest.mark.parametrize("fail_outer", [None, "3"])
def test_distributed_rank_failure_ends_every_rank(monkeypatch, fail_outer):
    """A rank that fails (SVM355_DECOMP_FAIL_RANK; before the first selection, or mid-solve at outer
    iteration SVM355_DECOMP_FAIL_OUTER) while the others wait in the solve's candidate all-gather: the
    group's abort ends every rank with the error instead of a hang, and the loopback group stays usable
    for the next fit."""
    from svm355._native import NativeError
    from svm355.parallel.decomp import DistributedDecompSVC
    from svm355.parallel.rccl import DeviceGroup

    tr = synthetic_mnist(4000, seed=95).compact()
    g = DeviceGroup(2, "loopback")
    try:
        monkeypatch.setenv("SVM355_DECOMP_FAIL_RANK", "1")
        if fail_outer:
            monkeypatch.setenv("SVM355_DECOMP_FAIL_OUTER", fail_outer)
        t0 = time.perf_counter()
        with pytest.raises(NativeError, match="injected failure"):
            DistributedDecompSVC(2, group=g).fit(tr.X, tr.y)
        assert time.perf_counter() - t0 < 60
        monkeypatch.delenv("SVM355_DECOMP_FAIL_RANK")
        monkeypatch.delenv("SVM355_DECOMP_FAIL_OUTER", raising=False)
        m = DistributedDecompSVC(2, group=g).fit(tr.X, tr.y)
    finally:
        g.close()
    one = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    assert m.stop_reason_ == "converged" and m.b_ == one.b_
    np.testing.assert_array_equal(m.alpha_, one.alpha_)


def test_column_cache_leaves_the_device_to_torch():
    """the decomposition's column cache (a grow-only slab of the context, outside PyTorch's
    allocator) takes at most a quarter of the HBM, and a later torch allocation that needs that memory
    gets it: ``ops.device.device_empty`` hands the library's caches back on an out-of-memory error."""
    import ctypes

    from svm355.ops import device as D

    tr = synthetic_mnist(250000, seed=3).compact()
    m = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)
    assert m.stop_reason_ == "converged"
    ctx = D.DeviceContext.get("cuda:0")
    slab = ctypes.c_int64(0)
    assert ctx.lib.svmd_cache_bytes(ctx.handle, None, ctypes.byref(slab)) == 0
    torch.cuda.empty_cache()  # no cached torch blocks: an allocation beyond `free` must come from the slab
    free, total = torch.cuda.mem_get_info(0)
    assert 0 < slab.value <= total // 4  # the cache ran (250k rows outgrow the last-level cache), capped
    need = free + slab.value // 2  # more than is free: only the slab's memory makes it fit
    t = D.device_empty(need // 8, torch.float64, "cuda:0")
    assert ctx.lib.svmd_cache_bytes(ctx.handle, None, ctypes.byref(slab)) == 0 and slab.value == 0
    del t
    torch.cuda.empty_cache()
    m2 = SVC(device="cuda:0", solver="decomp").fit(tr.X, tr.y)  # the cache is rebuilt on demand
    assert m2.b_ == m.b_


def test_scale_cli_decomp_rehearsal_times_every_rank_alone(tmp_path):
    """``python -m svm355 scale`` (the mpirun -np P sweep) defaults to the distributed decomposition; on
    one GPU (--transport loopback) every rank's device work per outer iteration is timed alone
    (SVM355_CASCADE_SERIAL_SOLVES), so each P's critical path is measured, and every P's model is the
    one-GPU model bit for bit."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    js = tmp_path / "s.json"
    r = subprocess.run([sys.executable, "-m", "svm355", "scale", "--transport", "loopback", "--ranks", "1,2,4",
                        "--sizes", "6000", "--test-rows", "500", "--repeats", "1", "--warmup", "0", "--json", str(js)],
                       cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    s = json.loads(js.read_text())
    rows = s["sizes"][0]["rows"]
    assert [x["P"] for x in rows] == [1, 2, 4]
    for x in rows:
        assert x["bit_identical_to_1gpu"] is True
    for x in rows[1:]:
        solo = x["solo"]
        assert solo and solo["outer_iterations"] >= 1 and len(solo["rank_select_ms"]) == x["P"]
        assert 0 < solo["select_ms"] + solo["rest_ms"] == pytest.approx(solo["critical_path_ms"])
        assert x["critical_path_solve_ms"] == solo["critical_path_ms"]
