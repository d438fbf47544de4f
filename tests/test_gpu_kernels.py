"""gfx950 kernels vs plain fp64 references, and the device SMO vs the CPU oracle.

Numerics tests compare each HIP kernel with a PyTorch/numpy fp64 computation of the same op; the
device SMO is checked bit-for-bit against the CPU oracle when both run on the same kernel matrix.
"""

import numpy as np
import pytest
import torch

from svm355 import SVC, SVMParams
from svm355.ops import cpu as C
from svm355.utils.data import MinMaxScaler, synthetic_mnist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from svm355.ops import device as D

    assert D.available(), "GPU visible but the HIP device library did not load"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def D():
    from svm355.ops import device as D

    return D


@pytest.fixture(scope="module")
def mn_data():
    return synthetic_mnist(1500, seed=5), synthetic_mnist(500, seed=5, offset=1500)


def test_native_library_is_loaded(dev):
    from svm355 import _native as N

    assert N._hip is not None
    with open("/proc/self/maps") as f:
        maps = f.read()
    assert "libsvm355_hip.so" in maps


def test_minmax_scale_norms(dev, D, mn_data):
    tr, _ = mn_data
    X = tr.X[:777].copy()
    X[:, 5] = 3.0  # constant column
    Xd = D.upload_rows(X, dev)
    assert Xd.shape == (777, 784) and torch.all(Xd[:, 784:] == 0)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    sc = MinMaxScaler().fit(X)
    np.testing.assert_array_equal(mn.cpu().numpy(), sc.min_)
    np.testing.assert_array_equal(mx.cpu().numpy(), sc.max_)
    Xs = sc.transform(X)
    np.testing.assert_array_equal(Xd[:, :784].cpu().numpy(), Xs)  # true division: bit-identical
    np.testing.assert_allclose(sqn.cpu().numpy(), (Xs ** 2).sum(1), rtol=1e-13)
    # test data with the training statistics
    Xq = D.upload_rows(X[:50] * 1.1, dev)
    D.minmax_scale_(Xq, 784, mn, mx)
    np.testing.assert_array_equal(Xq[:, :784].cpu().numpy(), sc.transform(X[:50] * 1.1))


def test_minmax_odd_width(dev, D):
    rng = np.random.default_rng(0)
    X = rng.normal(size=(1000, 37))
    Xd = D.upload_rows(X, dev)
    assert Xd.shape[1] == 48
    mn, mx = D.minmax(Xd, 37)
    np.testing.assert_array_equal(mn.cpu().numpy(), X.min(0))
    np.testing.assert_array_equal(mx.cpu().numpy(), X.max(0))


@pytest.mark.parametrize("m,n,d", [(300, 257, 784), (128, 128, 16), (1, 5, 33), (517, 1029, 100)])
def test_rbf_gram_vs_fp64_reference(dev, D, m, n, d):
    rng = np.random.default_rng(m + n + d)
    A = rng.uniform(0, 1, size=(m, d))
    B = rng.uniform(0, 1, size=(n, d))
    gamma = 0.5 / d
    Ad, Bd = D.upload_rows(A, dev), D.upload_rows(B, dev)
    K = D.rbf_gram(Ad, D.row_norms(Ad, d), Bd, D.row_norms(Bd, d), gamma)
    ref = C.rbf_matrix(A, B, gamma)
    np.testing.assert_allclose(K[:, :n].cpu().numpy(), ref, rtol=0, atol=2e-14)


def test_rbf_gram_symmetric_diag_exact(dev, D, mn_data):
    tr, _ = mn_data
    X = MinMaxScaler().fit_transform(tr.X[:600])
    Xd = D.upload_rows(X, dev)
    nrm = D.row_norms(Xd, 784)
    K = D.rbf_gram(Xd, nrm, Xd, nrm, 0.00125, symmetric=True)[:, :600].cpu().numpy()
    assert np.all(np.diag(K) == 1.0)
    np.testing.assert_array_equal(K, K.T)  # exactly symmetric
    np.testing.assert_allclose(K, C.rbf_matrix(X, X, 0.00125), rtol=0, atol=1e-13)


def test_gather_rows(dev, D):
    X = torch.arange(40 * 32, dtype=torch.float64, device=dev).reshape(40, 32)
    idx = torch.tensor([5, 0, 39, 5], device=dev)
    assert torch.equal(D.gather_rows(X, idx), X[idx])


@pytest.fixture
def smo_mode(request, monkeypatch):
    mode, wg = request.param
    monkeypatch.setenv("SVM355_SMO", mode)
    if wg:
        monkeypatch.setenv("SVM355_PSMO_WG", str(wg))
    return request.param


@pytest.mark.parametrize("smo_mode", [("persistent", None), ("persistent", 1), ("persistent", 3), ("graph", None),
                                      ("single", None)],
                         indirect=True, ids=["persistent", "persistent-G1", "persistent-G2", "graph", "single"])
def test_device_smo_bit_identical_to_oracle_on_same_gram(dev, D, mn_data, smo_mode):
    tr, _ = mn_data
    X = MinMaxScaler().fit_transform(tr.X[:900])
    y = tr.y[:900]
    p = SVMParams(n_threads=8)
    K = C.rbf_matrix(X, X, p.gamma, 8)
    a_cpu, r_cpu, t_cpu = C.smo_train_gram(K, y, p, trace_cap=200000)
    Kd = torch.from_numpy(K).to(dev)
    yd = torch.from_numpy(y).to(dev)
    ad = torch.zeros(900, dtype=torch.float64, device=dev)
    r_gpu, t_gpu = D.smo(Kd, yd, ad, p, trace_cap=200000)
    assert r_gpu.iterations == r_cpu.iterations
    assert r_gpu.stop_reason == r_cpu.stop_reason == "converged"
    np.testing.assert_array_equal(t_gpu, t_cpu)
    np.testing.assert_array_equal(ad.cpu().numpy(), a_cpu)
    assert r_gpu.b == r_cpu.b


@pytest.mark.parametrize("n,xcd", [(900, "1"), (900, "0"), (9000, "1"), (20000, "1"), (20000, "0")],
                         ids=["xcd-900", "device-900", "xcd-9k", "xcd-20k", "device-20k"])
def test_device_wss2_bit_identical_to_oracle_on_same_gram(dev, D, monkeypatch, n, xcd):
    """Opt-in second-order selection (svm_params.wss = 2): the persistent solver's second exchange
    picks the same j as the CPU oracle on the same (device-built) Gram -- identical (i, j) traces,
    alphas and b -- in fewer iterations than first order."""
    monkeypatch.setenv("SVM355_PSMO_XCD", xcd)
    tr = synthetic_mnist(n, seed=31)
    Xd = D.upload_rows(tr.compact().X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    Kd, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    K = Kd[:, :n].contiguous().cpu().numpy()
    yd = torch.from_numpy(tr.y).to(dev)
    p2 = SVMParams(n_threads=8, wss=2)
    a_cpu, r_cpu, t_cpu = C.smo_train_gram(K, tr.y, p2, trace_cap=200000)
    ad = torch.zeros(n, dtype=torch.float64, device=dev)
    r_gpu, t_gpu = D.smo(Kd, yd, ad, p2, n=n, trace_cap=200000)
    assert r_gpu.stop_reason == r_cpu.stop_reason == "converged"
    assert r_gpu.iterations == r_cpu.iterations
    np.testing.assert_array_equal(t_gpu, t_cpu)
    np.testing.assert_array_equal(ad.cpu().numpy(), a_cpu)
    assert r_gpu.b == r_cpu.b
    a1 = torch.zeros(n, dtype=torch.float64, device=dev)
    r1, _ = D.smo(Kd, yd, a1, SVMParams(), n=n)
    assert r_gpu.iterations < r1.iterations


def test_persistent_vs_graph_many_workgroups(dev, D, monkeypatch):
    """Many workgroups (G = 40 at n = 20000): both device paths bit-identical."""
    tr = synthetic_mnist(20000, seed=9)
    Xd = D.upload_rows(tr.X, dev)
    _, _, sqn = D.minmax_scale_(Xd, 784)
    K = D.rbf_gram(Xd, sqn, Xd, sqn, 0.00125, symmetric=True)
    yd = torch.from_numpy(tr.y).to(dev)
    out = {}
    for mode in ("persistent", "graph"):
        monkeypatch.setenv("SVM355_SMO", mode)
        monkeypatch.setenv("SVM355_PSMO_WG", "64")
        a = torch.zeros(tr.n, dtype=torch.float64, device=dev)
        r, trc = D.smo(K, yd, a, SVMParams(), n=tr.n, trace_cap=1000000)
        out[mode] = (r, trc, a.cpu().numpy())
    (r1, t1, a1), (r2, t2, a2) = out["persistent"], out["graph"]
    assert r1.iterations == r2.iterations and r1.b == r2.b and r1.stop_reason == "converged"
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(a1, a2)


@pytest.mark.parametrize("n", [3000, 7000])
def test_single_workgroup_smo_matches_persistent(dev, D, monkeypatch, n):
    """The single-workgroup solver (E = 4 and 8 register elements) follows the persistent trajectory."""
    tr = synthetic_mnist(n, seed=11)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    out = {}
    for mode in ("single", "persistent"):
        monkeypatch.setenv("SVM355_SMO", mode)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        r, trc = D.smo(K, yd, a, SVMParams(), n=n, trace_cap=200000)
        out[mode] = (r, trc, a.cpu().numpy())
    (r1, t1, a1), (r2, t2, a2) = out["single"], out["persistent"]
    assert r1.iterations == r2.iterations and r1.b == r2.b and r1.stop_reason == "converged"
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(a1, a2)


@pytest.mark.parametrize("n", [5000, 20000])
def test_xcd_local_persistent_smo_matches_graph(dev, D, monkeypatch, n):
    """XCD-local persistent solver (records through one XCD's L2) follows the graph-replay trajectory."""
    tr = synthetic_mnist(n, seed=13)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    out = {}
    for mode, xcd in (("persistent", "1"), ("graph", "0")):
        monkeypatch.setenv("SVM355_SMO", mode)
        monkeypatch.setenv("SVM355_PSMO_XCD", xcd)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        r, trc = D.smo(K, yd, a, SVMParams(), n=n, trace_cap=200000)
        out[mode] = (r, trc, a.cpu().numpy())
    (r1, t1, a1), (r2, t2, a2) = out["persistent"], out["graph"]
    assert r1.iterations == r2.iterations and r1.b == r2.b and r1.stop_reason == "converged"
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(a1, a2)


def test_headline_shape_60k_default_solver_equals_graph_replay(dev, D, monkeypatch):
    """The bench's exact shape: n = 60000 MNIST-shaped rows, resident exact-integer Gram, the default
    solver (XCD-local persistent, 512-thread workgroups x 4 elements) against the two-kernel graph
    replay: identical (i_high, i_low) traces, alphas and b; and SVC.fit (what bench.py times)
    reports that solve's iterations and b."""
    n = 60000
    tr = synthetic_mnist(n, seed=2024).compact()
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, path = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    assert path == "int8-exact"
    yd = torch.from_numpy(tr.y).to(dev)
    out = {}
    for mode in ("auto", "graph"):
        monkeypatch.setenv("SVM355_SMO", mode)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        r, trc = D.smo(K, yd, a, SVMParams(), n=n, trace_cap=20000)
        out[mode] = (r, trc, a.cpu().numpy())
    monkeypatch.delenv("SVM355_SMO")
    (r1, t1, a1), (r2, t2, a2) = out["auto"], out["graph"]
    assert r1.stop_reason == "converged" and r1.iterations == 12793  # the README / BENCH headline solve
    assert r1.iterations == r2.iterations and r1.b == r2.b
    assert len(t1) == r1.iterations - 1
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(a1, a2)
    del K
    m = SVC(device="cuda:0", solver="smo").fit(tr.X, tr.y)
    assert m.n_iter_ == r1.iterations and m.b_ == r1.b
    assert m.timings_["gram_path"] == "int8-exact" and m.timings_["kcache"] == "full"
    assert m.timings_.get("rows") == "uint8"  # bench.py's byte path (SVC._fit_cuda_u8)


def test_device_smo_warm_start_bit_identical(dev, D, mn_data):
    tr, _ = mn_data
    X = MinMaxScaler().fit_transform(tr.X[:700])
    y = tr.y[:700]
    p = SVMParams(n_threads=8)
    K = C.rbf_matrix(X, X, p.gamma, 8)
    a_cold, _, _ = C.smo_train_gram(K, y, p)
    a0 = a_cold * 0.5
    a_cpu, r_cpu, _ = C.smo_train_gram(K, y, p, alpha=a0, warm=True)
    ad = torch.from_numpy(a0.copy()).to(dev)
    r_gpu, _ = D.smo(torch.from_numpy(K).to(dev), torch.from_numpy(y).to(dev), ad, p, warm=True)
    assert r_gpu.iterations == r_cpu.iterations
    np.testing.assert_array_equal(ad.cpu().numpy(), a_cpu)
    assert r_gpu.b == r_cpu.b


def test_device_smo_stop_reasons(dev, D, mn_data):
    tr, _ = mn_data
    X = MinMaxScaler().fit_transform(tr.X[:300])
    K = torch.from_numpy(C.rbf_matrix(X, X, 0.00125)).to(dev)
    y = torch.from_numpy(tr.y[:300]).to(dev)
    a = torch.zeros(300, dtype=torch.float64, device=dev)
    r, tr_ = D.smo(K, y, a, SVMParams(max_iter=7), trace_cap=50)
    assert r.stop_reason == "max_iter" and r.iterations == 8 and tr_.shape == (7, 2)
    r, _ = D.smo(K, torch.ones(300, dtype=torch.int32, device=dev), a, SVMParams())
    assert r.stop_reason == "no_candidate"


def test_device_train_matches_oracle(dev, D, mn_data):
    """Full device path (MFMA Gram + SMO): same optimum as the oracle (K differs in the last ulps)."""
    tr, _ = mn_data
    sc = MinMaxScaler().fit(tr.X)
    a_cpu, r_cpu, _ = C.smo_train(sc.transform(tr.X), tr.y, SVMParams(n_threads=8))
    Xd = D.upload_rows(tr.X, dev)
    _, _, sqn = D.minmax_scale_(Xd, 784)
    ad = torch.zeros(tr.n, dtype=torch.float64, device=dev)
    r_gpu, tm = D.train(Xd, sqn, torch.from_numpy(tr.y).to(dev), ad, SVMParams())
    a_gpu = ad.cpu().numpy()
    assert r_gpu.stop_reason == "converged"
    assert abs(r_gpu.iterations - r_cpu.iterations) <= max(5, r_cpu.iterations // 50)
    s_cpu = set(np.flatnonzero(a_cpu > 1e-8).tolist())
    s_gpu = set(np.flatnonzero(a_gpu > 1e-8).tolist())
    assert len(s_cpu ^ s_gpu) <= 2
    assert abs(r_gpu.b - r_cpu.b) < 1e-6 * max(1, abs(r_cpu.b))
    np.testing.assert_allclose(a_gpu, a_cpu, atol=1e-6)


def test_decision_vs_fp64_reference(dev, D, mn_data):
    tr, te = mn_data
    sc = MinMaxScaler().fit(tr.X)
    Xs, Xq = sc.transform(tr.X[:333]), sc.transform(te.X[:211])
    rng = np.random.default_rng(3)
    coef = rng.uniform(-10, 10, 333)
    Xsd, Xqd = D.upload_rows(Xs, dev), D.upload_rows(Xq, dev)
    out = D.decision(Xsd, D.row_norms(Xsd, 784), torch.from_numpy(coef).to(dev), Xqd, D.row_norms(Xqd, 784),
                     0.00125, 0.75).cpu().numpy()
    ref = C.rbf_matrix(Xq, Xs, 0.00125) @ coef - 0.75
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-11)


@pytest.mark.parametrize("m", [1, 255, 257, 10000, 300001])
def test_count_correct_vs_numpy(dev, D, m):
    """Device accuracy count (predict flag + reduce_sum) for both sign rules, exact zeros included."""
    rng = np.random.default_rng(m)
    dec = rng.normal(size=m)
    dec[rng.random(m) < 0.05] = 0.0
    y = np.where(rng.random(m) < 0.5, 1, -1).astype(np.int32)
    dd = torch.from_numpy(dec).to(dev)
    for zp in (False, True):
        pred = np.where(dec >= 0 if zp else dec > 0, 1, -1)
        assert D.count_correct(dd, y, zp) == int(np.sum(pred == y))


def test_svc_cuda_matches_cpu(dev, mn_data):
    tr, te = mn_data
    g = SVC(device="cuda", solver="smo").fit(tr.X, tr.y)
    c = SVC(device="cpu", n_threads=8).fit(tr.X, tr.y)
    assert abs(g.b_ - c.b_) < 1e-6 * max(1, abs(c.b_))
    assert len(set(g.support_.tolist()) ^ set(c.support_.tolist())) <= 2
    np.testing.assert_allclose(g.decision_function(te.X), c.decision_function(te.X), atol=1e-5)
    assert g.score(te.X, te.y) == c.score(te.X, te.y)


def test_svc_cuda_save_load(tmp_path, dev, mn_data):
    tr, te = mn_data
    g = SVC(device="cuda").fit(tr.X, tr.y)
    g.save(tmp_path / "m")
    g2 = SVC.load(tmp_path / "m", device="cuda")
    np.testing.assert_allclose(g2.decision_function(te.X), g.decision_function(te.X), atol=1e-12)


# ---------------------------------------------------------------- exact-integer Gram (igram.hip)
def _exact_rbf(P: np.ndarray, mn: np.ndarray, mx: np.ndarray, gamma: float) -> np.ndarray:
    """K from the integer pixels: dist = sum_j (q_aj - q_bj)^2 / r_j^2 with exact integer differences."""
    r = mx - mn
    r = np.where(r < 1e-12, 1.0, r)
    Q = P - mn  # exact integers
    w = 1.0 / (r * r)
    d2 = np.zeros((P.shape[0], P.shape[0]))
    for j in range(P.shape[1]):  # per-column exact squared differences, weighted in fp64
        dq = Q[:, j][:, None] - Q[:, j][None, :]
        d2 += w[j] * dq * dq
    return np.exp(-gamma * d2)


def _int_data(n, d, seed, ranges):
    rng = np.random.default_rng(seed)
    hi = rng.choice(ranges, size=d)
    P = np.floor(rng.random((n, d)) * (hi + 1)).astype(np.float64)
    P[0] = 0.0
    P[1] = hi  # every column attains [0, hi]
    return P


@pytest.mark.parametrize("n,d,ranges,seed", [
    (700, 784, [255], 1),                  # no correction columns (kc = 0)
    (1031, 784, [255] * 9 + [254, 200], 2),  # ~18% correction columns
    (300, 100, [255] * 6 + [17, 3, 1], 3),  # several distinct ranges, small d
    (129, 40, [100], 4),                   # base range != 255
    (777, 300, [255] * 8 + [254, 127, 2, 85, 253], 5),  # ranges merged into 255 / 254 (divisors), 253 apart
])
def test_int_gram_matches_exact(dev, D, n, d, ranges, seed):
    P = _int_data(n, d, seed, ranges)
    P[:, 3] = 7.0  # constant column
    Xd = D.upload_rows(P, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, d)
    gamma = 0.00125 * 784 / d
    K, path = D.rbf_gram_sym(Xd, sqn, gamma, mn=mn, mx=mx, gram="int")
    assert path == "int8-exact"
    Kh = K[:, :n].cpu().numpy()
    ref = _exact_rbf(P, P.min(0), P.max(0), gamma)
    assert np.abs(Kh - ref).max() <= 2e-15
    np.testing.assert_array_equal(np.diag(Kh), 1.0)
    np.testing.assert_array_equal(Kh, Kh.T)  # mirror stores
    Kf, pf = D.rbf_gram_sym(Xd, sqn, gamma, mn=mn, mx=mx, gram="fp64")
    assert pf == "fp64"
    assert np.abs(Kf[:, :n].cpu().numpy() - ref).max() <= 1e-13


def test_int_gram_falls_back_on_real_valued_data(dev, D):
    rng = np.random.default_rng(9)
    X = rng.random((300, 50)) * 3.0
    Xd = D.upload_rows(X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 50)
    K, path = D.rbf_gram_sym(Xd, sqn, 0.1, mn=mn, mx=mx, gram="auto")
    assert path == "fp64"
    with pytest.raises(Exception):
        D.rbf_gram_sym(Xd, sqn, 0.1, mn=mn, mx=mx, gram="int")


def test_near_integer_rows_take_the_fp64_gram(dev, mn_data):
    """Values a few 1e-7 off an integer are real-valued data: the auto Gram must not round them onto
    the exact-integer path (igram.hip quantisation tolerance is ~64 ulp of the pixel range)."""
    tr, _ = mn_data
    X = tr.X[:600].copy()
    col = int(np.argmax(X.max(0) - X.min(0)))
    inner = np.flatnonzero((X[:, col] > X[:, col].min()) & (X[:, col] < X[:, col].max()))
    assert len(inner) > 3
    X[inner[::3], col] += 4e-7  # e.g. 3.0000004; min / max (and so the range plan) stay integers
    a = SVC(device="cuda:0", solver="smo").fit(X, tr.y[:600])
    assert a.timings_["gram_path"] == "fp64"
    b = SVC(device="cuda:0", solver="smo").fit(tr.X[:600], tr.y[:600])
    assert b.timings_["gram_path"] == "int8-exact"


def test_decision_int_block_is_the_grams_columns(dev, D):
    """svmd_decision_int (the cascade's warm-start check): the exact-integer block K(X, X[0:nz]) is
    bit-identical to those columns of the resident exact-integer Gram (unit coefficient vectors pick
    single columns), and its GEMV matches K[:, :nz] @ coef; real-valued rows are refused (None)."""
    n, nz = 3000, 700
    tr = synthetic_mnist(n, seed=41)
    Xd = D.upload_rows(tr.compact().X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, path = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    assert path == "int8-exact"
    for j in (0, 129, nz - 1):
        e = torch.zeros(nz, dtype=torch.float64, device=dev)
        e[j] = 1.0
        out = D.decision_int(Xd, 784, mn, mx, e, 0.00125)
        assert out is not None and torch.equal(out, K[:n, j])
    g = torch.Generator(device="cpu").manual_seed(3)
    coef = torch.randn(nz, dtype=torch.float64, generator=g).to(dev)
    out = D.decision_int(Xd, 784, mn, mx, coef, 0.00125)
    torch.testing.assert_close(out, K[:n, :nz] @ coef, rtol=1e-13, atol=1e-11)
    rng = np.random.default_rng(2)
    Xr = D.upload_rows(rng.normal(size=(300, 20)), dev)
    mnr, mxr, _ = D.minmax_scale_(Xr, 20)
    assert D.decision_int(Xr, 20, mnr, mxr, coef[:50], 0.05) is None


def test_svc_int_gram_matches_fp64_gram(dev, mn_data):
    tr, te = mn_data
    a = SVC(device="cuda:0", gram="int").fit(tr.X, tr.y)
    b = SVC(device="cuda:0", gram="fp64").fit(tr.X, tr.y)
    c = SVC(device="cpu").fit(tr.X, tr.y)
    assert a.timings_["gram_path"] == "int8-exact" and b.timings_["gram_path"] == "fp64"
    assert a.stop_reason_ == "converged"
    assert set(a.support_.tolist()) == set(c.support_.tolist())
    assert abs(a.b_ - c.b_) <= 1e-7 * max(1.0, abs(c.b_))
    assert abs(a.b_ - b.b_) <= 1e-7 * max(1.0, abs(c.b_))
    np.testing.assert_array_equal(a.predict(te.X), c.predict(te.X))


def test_upload_u8_rows_equal_fp64_upload(dev, D, mn_data):
    tr, _ = mn_data
    Xc = tr.compact().X
    assert Xc.dtype == np.uint8
    for ld in (None, 800):
        a = D.upload_rows(Xc[:517], dev, ld)
        b = D.upload_rows(tr.X[:517], dev, ld)
        assert a.dtype == torch.float64 and a.shape == b.shape == (517, ld or 784)
        assert torch.equal(a, b)  # includes the zero padding columns


def test_svc_u8_rows_bit_identical_to_fp64_rows(dev, mn_data):
    tr, te = mn_data
    a = SVC(device="cuda:0", solver="smo").fit(tr.compact().X, tr.y)
    b = SVC(device="cuda:0", solver="smo").fit(tr.X, tr.y)
    assert a.b_ == b.b_ and a.n_iter_ == b.n_iter_
    np.testing.assert_array_equal(a.alpha_, b.alpha_)
    np.testing.assert_array_equal(a.decision_function(te.compact().X), b.decision_function(te.X))


def test_svc_byte_path_equals_fp64_row_path(dev, mn_data, monkeypatch):
    """uint8 rows take the byte path (min/max, quantisation and Gram straight from the bytes, only the
    SVs widened; SVC._fit_cuda_u8); with SVM355_U8_TRAIN=0 the same rows go through the FP64-row path.
    The models -- alphas, b, SV rows and norms, decisions -- must be identical bit for bit."""
    tr, te = mn_data
    Xc = tr.compact().X
    a = SVC(device="cuda:0", solver="smo").fit(Xc, tr.y)
    assert a.timings_.get("rows") == "uint8" and a.timings_["gram_path"] == "int8-exact"
    monkeypatch.setenv("SVM355_U8_TRAIN", "0")
    b = SVC(device="cuda:0", solver="smo").fit(Xc, tr.y)
    assert "rows" not in b.timings_
    assert a.b_ == b.b_ and a.n_iter_ == b.n_iter_
    np.testing.assert_array_equal(a.alpha_, b.alpha_)
    assert torch.equal(a._dev["Xs"], b._dev["Xs"]) and torch.equal(a._dev["ns"], b._dev["ns"])
    assert torch.equal(a._dev["mn"], b._dev["mn"]) and torch.equal(a._dev["mx"], b._dev["mx"])
    np.testing.assert_array_equal(a.decision_function(te.compact().X), b.decision_function(te.compact().X))


# ---------------------------------------------------------------- on-demand row cache (rowcache.hip)
@pytest.mark.parametrize("cache_rows", [6, 64, 100000])
def test_row_cache_smo_bit_identical_to_full_gram(dev, D, cache_rows):
    """Row-cache SMO (tiny / small / unbounded cache) follows the full-Gram trajectory bit for bit."""
    n = 2500
    tr = synthetic_mnist(n, seed=21)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    yd = torch.from_numpy(tr.y).to(dev)
    K, path = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    assert path == "int8-exact"
    a_full = torch.zeros(n, dtype=torch.float64, device=dev)
    r_full, t_full = D.smo(K, yd, a_full, SVMParams(), n=n, trace_cap=100000)
    a_rows = torch.zeros(n, dtype=torch.float64, device=dev)
    ldc = (n + 1) // 2 * 2
    r_rows, info = D.train(Xd, sqn, yd, a_rows, SVMParams(), mn=mn, mx=mx, kcache="rows",
                           cache_bytes=cache_rows * ldc * 8, trace_cap=100000)
    assert info["kcache"] == "rows" and info["gram_path"] == "int8-exact"
    assert r_rows.iterations == r_full.iterations and r_rows.b == r_full.b
    assert r_rows.stop_reason == "converged"
    np.testing.assert_array_equal(info["trace"], t_full)
    np.testing.assert_array_equal(a_rows.cpu().numpy(), a_full.cpu().numpy())


@pytest.mark.parametrize("n,cache_rows", [(2500, 64), (40000, 512)])
def test_persistent_row_cache_equals_graph_row_cache(dev, D, monkeypatch, n, cache_rows):
    """The persistent row-cache solver (replicated LDS directory, slices filled on a miss) against
    the replayed select / step graph: the same trace, alphas and b; at n = 40k the device-wide team
    has 40 workgroups and a 512-row cache that evicts."""
    tr = synthetic_mnist(n, seed=23)
    Xd = D.upload_rows(tr.compact().X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    yd = torch.from_numpy(tr.y).to(dev)
    ldc = (n + 1) // 2 * 2
    out = {}
    for mode in ("persistent", "graph"):
        monkeypatch.setenv("SVM355_RC_SMO", mode)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        r, info = D.train(Xd, sqn, yd, a, SVMParams(), mn=mn, mx=mx, kcache="rows", cache_bytes=cache_rows * ldc * 8,
                          trace_cap=200000)
        out[mode] = (r, info["trace"], a.cpu().numpy())
    (r1, t1, a1), (r2, t2, a2) = out["persistent"], out["graph"]
    assert r1.stop_reason == "converged" and r1.iterations == r2.iterations and r1.b == r2.b
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(a1, a2)


def test_row_cache_wide_teams_follow_the_same_trajectory(dev, D, monkeypatch):
    """Teams of more than 64 workgroups (each sweep lane merges two or four records under wave_arg's
    order, smo.hip persist_solve<..., RPL>): n = 70k as 35 x E=4 (one record per lane), 69 x E=2
    (SVM355_RC_MAXG=128: two) and 137 x E=1 (=256: four) -- the same trace, alphas and b."""
    n = 70000
    tr = synthetic_mnist(n, seed=24)
    Xd = D.upload_rows(tr.compact().X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    yd = torch.from_numpy(tr.y).to(dev)
    out = {}
    for maxg in ("64", "128", "256"):
        monkeypatch.setenv("SVM355_RC_MAXG", maxg)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        r, info = D.train(Xd, sqn, yd, a, SVMParams(), mn=mn, mx=mx, kcache="rows", trace_cap=200000)
        out[maxg] = (r, info["trace"], a.cpu().numpy())
    r0, t0, a0 = out["64"]
    assert r0.stop_reason == "converged"
    for maxg in ("128", "256"):
        r, t, a = out[maxg]
        assert r.iterations == r0.iterations and r.b == r0.b, maxg
        np.testing.assert_array_equal(t, t0)
        np.testing.assert_array_equal(a, a0)


@pytest.mark.parametrize("n,cache_rows", [(2500, 6), (2500, 64), (40000, 512)])
def test_row_cache_wss2_bit_identical_to_resident_gram(dev, D, n, cache_rows):
    """Opt-in second-order selection on the persistent row-cache solver: row i_high is looked up before
    the second exchange and row j after it, with i_high's slot kept (a 6-row cache evicts every
    iteration) -- the same (i, j) trace, alphas and b as second order on the resident Gram."""
    tr = synthetic_mnist(n, seed=25)
    Xd = D.upload_rows(tr.compact().X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    yd = torch.from_numpy(tr.y).to(dev)
    K, path = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    assert path == "int8-exact"
    p2 = SVMParams(wss=2)
    a_full = torch.zeros(n, dtype=torch.float64, device=dev)
    r_full, t_full = D.smo(K, yd, a_full, p2, n=n, trace_cap=200000)
    del K
    ldc = (n + 1) // 2 * 2
    a_rows = torch.zeros(n, dtype=torch.float64, device=dev)
    r_rows, info = D.train(Xd, sqn, yd, a_rows, p2, mn=mn, mx=mx, kcache="rows", cache_bytes=cache_rows * ldc * 8,
                           trace_cap=200000)
    assert r_rows.stop_reason == r_full.stop_reason == "converged"
    assert r_rows.iterations == r_full.iterations and r_rows.b == r_full.b
    np.testing.assert_array_equal(info["trace"], t_full)
    np.testing.assert_array_equal(a_rows.cpu().numpy(), a_full.cpu().numpy())


def test_row_cache_wss2_needs_integer_rows(dev, D):
    """Second order on real-valued rows (FP64 on-demand rows, graph-replayed solver) is refused loudly."""
    rng = np.random.default_rng(6)
    X = rng.normal(size=(300, 20))
    y = np.where(X[:, 0] > 0, 1, -1).astype(np.int32)
    with pytest.raises(Exception, match="second-order"):
        SVC(device="cuda:0", kcache="rows", wss="second").fit(X, y)


def test_row_cache_warm_start_bit_identical(dev, D):
    n = 1800
    tr = synthetic_mnist(n, seed=22)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    yd = torch.from_numpy(tr.y).to(dev)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    a0 = torch.zeros(n, dtype=torch.float64, device=dev)
    D.smo(K, yd, a0, SVMParams(), n=n)
    a0 = a0 * 0.5
    a_full = a0.clone()
    r_full, _ = D.smo(K, yd, a_full, SVMParams(), n=n, warm=True)
    a_rows = a0.clone()
    r_rows, _ = D.train(Xd, sqn, yd, a_rows, SVMParams(), warm=True, mn=mn, mx=mx, kcache="rows",
                        cache_bytes=40 * n * 8)
    assert r_rows.iterations == r_full.iterations and r_rows.b == r_full.b
    np.testing.assert_array_equal(a_rows.cpu().numpy(), a_full.cpu().numpy())


def test_row_cache_fp64_rows_match_oracle(dev, D):
    """Real-valued features: FP64 kernel rows computed on demand; same optimum as the CPU oracle."""
    rng = np.random.default_rng(5)
    n = 1200
    X = rng.normal(size=(n, 30))
    y = np.where(X[:, 0] + 0.5 * X[:, 1] ** 2 + 0.3 * rng.normal(size=n) > 0.4, 1, -1).astype(np.int32)
    c = SVC(device="cpu", gamma=0.05, C=2.0).fit(X, y)
    g = SVC(device="cuda:0", gamma=0.05, C=2.0, kcache="rows").fit(X, y)
    assert g.timings_["kcache"] == "rows" and g.timings_["gram_path"] == "fp64"
    assert g.stop_reason_ == "converged"
    assert set(g.support_.tolist()) == set(c.support_.tolist())
    assert abs(g.b_ - c.b_) <= 1e-6 * max(1.0, abs(c.b_))


def test_ovr_multiclass_gpu_matches_cpu(dev):
    from svm355 import OneVsRestSVC

    tr = synthetic_mnist(1500, seed=31)
    te = synthetic_mnist(400, seed=31, offset=1500)
    g = OneVsRestSVC(device="cuda:0", solver="batched").fit(tr.X, tr.labels)
    c = OneVsRestSVC(device="cpu").fit(tr.X, tr.labels)
    assert g.timings_["gram_path"] == "int8-exact"
    assert all(s == "converged" for s in g.stop_reasons_)
    np.testing.assert_array_equal(g.support_, c.support_)
    np.testing.assert_allclose(g.intercepts_b_, c.intercepts_b_, rtol=0, atol=1e-7)
    np.testing.assert_array_equal(g.predict(te.X), c.predict(te.X))


def test_ovr_distributed_threads_gpu_equals_single_rank(dev):
    """Two ranks on the one GPU (thread transport): each solves its classes on its own Gram; the
    all-reduced model equals the single-rank device fit exactly."""
    from svm355 import OneVsRestSVC
    from svm355.parallel.transport import run_threads

    tr = synthetic_mnist(1200, seed=32)
    one = OneVsRestSVC(device="cuda:0").fit(tr.X, tr.labels)

    def fn(t):
        m = OneVsRestSVC(device="cuda:0").fit(tr.X, tr.labels, transport=t)
        return m.support_, m.dual_coef_, m.intercepts_b_, m.n_iter_

    for sup, coef, b, it in run_threads(2, fn, device_for_rank=lambda r: torch.device("cuda:0")):
        np.testing.assert_array_equal(sup, one.support_)
        np.testing.assert_array_equal(coef, one.dual_coef_)
        np.testing.assert_array_equal(b, one.intercepts_b_)
        np.testing.assert_array_equal(it, one.n_iter_)


@pytest.mark.parametrize("n", [1500, 5000, 26000])
def test_ovr_batched_xcd_teams_equal_per_class_solves(dev, n):
    """All classes in one launch (an XCD-local team per XCD pulling classes from a queue) gives the
    per-class persistent solves' results bit for bit; shapes cover 256-, 512- and 1024-thread teams."""
    from svm355 import OneVsRestSVC

    tr = synthetic_mnist(n, seed=33)
    b = OneVsRestSVC(device="cuda:0", solver="batched").fit(tr.X, tr.labels)
    s = OneVsRestSVC(device="cuda:0", solver="streams").fit(tr.X, tr.labels)
    assert b.timings_["smo_solver"] == "batched" and s.timings_["smo_solver"] == "streams"
    assert all(r == "converged" for r in b.stop_reasons_)
    np.testing.assert_array_equal(b.n_iter_, s.n_iter_)
    np.testing.assert_array_equal(b.intercepts_b_, s.intercepts_b_)
    np.testing.assert_array_equal(b.support_, s.support_)
    np.testing.assert_array_equal(b.dual_coef_, s.dual_coef_)


def test_ovr_second_order_batched_equals_per_class_solves(dev):
    """wss="second" in the batched one-launch solver (smo_multi_kernel<..., WSS2>) gives the per-class
    second-order persistent solves' models bit for bit, in fewer iterations than first order."""
    from svm355 import OneVsRestSVC

    tr = synthetic_mnist(6000, seed=35)
    X = tr.compact().X
    b = OneVsRestSVC(device="cuda:0", solver="batched", wss="second").fit(X, tr.labels)
    s = OneVsRestSVC(device="cuda:0", solver="streams", wss="second").fit(X, tr.labels)
    f = OneVsRestSVC(device="cuda:0", solver="batched").fit(X, tr.labels)
    assert b.timings_["smo_solver"] == "batched" and all(r == "converged" for r in b.stop_reasons_)
    np.testing.assert_array_equal(b.n_iter_, s.n_iter_)
    np.testing.assert_array_equal(b.intercepts_b_, s.intercepts_b_)
    np.testing.assert_array_equal(b.dual_coef_, s.dual_coef_)
    assert b.n_iter_.sum() < f.n_iter_.sum()


def test_ovr_byte_path_equals_fp64_row_path(dev, monkeypatch):
    """One-vs-rest on uint8 rows: the Gram straight from the device bytes (svmd_rbf_gram_u8) and SVs
    widened alone give the FP64-row path's models bit for bit (SVM355_U8_TRAIN=0 forces the latter)."""
    from svm355 import OneVsRestSVC

    tr = synthetic_mnist(3000, seed=34)
    te = synthetic_mnist(400, seed=34, offset=3000)
    X = tr.compact().X
    a = OneVsRestSVC(device="cuda:0", solver="batched").fit(X, tr.labels)
    monkeypatch.setenv("SVM355_U8_TRAIN", "0")
    b = OneVsRestSVC(device="cuda:0", solver="batched").fit(X, tr.labels)
    assert a.timings_["gram_path"] == b.timings_["gram_path"] == "int8-exact"
    np.testing.assert_array_equal(a.n_iter_, b.n_iter_)
    np.testing.assert_array_equal(a.intercepts_b_, b.intercepts_b_)
    np.testing.assert_array_equal(a.support_, b.support_)
    np.testing.assert_array_equal(a.dual_coef_, b.dual_coef_)
    assert torch.equal(a._dev_model["Xs"], b._dev_model["Xs"]) and torch.equal(a._dev_model["ns"], b._dev_model["ns"])
    np.testing.assert_array_equal(a.predict(te.compact().X), b.predict(te.compact().X))


def test_ovr_decomposition_equals_its_oracle_per_class(dev):
    """The GPU default one-vs-rest (solver="decomp": every class by the decomposition solver on the shared
    device rows, no Gram, classes on concurrent host threads) gives, class by class, the CPU decomposition
    oracle's alpha, b and iterations bit for bit (on the device's exact kernel values), the same from
    uint8 and FP64 host rows, and predicts like the batched pairwise solve."""
    from svm355 import OneVsRestSVC
    from svm355.ops import device as Dv

    tr = synthetic_mnist(2500, seed=36)
    te = synthetic_mnist(400, seed=36, offset=2500)
    Xb = tr.compact().X
    g = OneVsRestSVC(device="cuda:0").fit(Xb, tr.labels)
    f = OneVsRestSVC(device="cuda:0", solver="decomp").fit(tr.X, tr.labels)
    p = OneVsRestSVC(device="cuda:0", solver="batched").fit(Xb, tr.labels)
    assert g.timings_["smo_solver"] == "decomp" and g.timings_["gram_ms"] == 0.0
    assert all(s == "converged" for s in g.stop_reasons_)
    for a, b in ((g.support_, f.support_), (g.dual_coef_, f.dual_coef_), (g.intercepts_b_, f.intercepts_b_),
                 (g.n_iter_, f.n_iter_)):
        np.testing.assert_array_equal(a, b)
    Xu = Dv.upload_u8(Xb, torch.device("cuda:0"))
    mmd = torch.empty(2 * tr.d, dtype=torch.float64, device="cuda:0")
    mn, mx = Dv.minmax_u8(Xu, out=mmd)
    mm = mmd.cpu().numpy()
    K = Dv.rbf_gram_u8(Xu, 0.00125, mm[: tr.d].copy(), mm[tr.d:].copy())
    Kh = np.ascontiguousarray(K[: tr.n, : tr.n].cpu().numpy())
    del K
    Dv.release_gram_buffers()
    coef = np.zeros((tr.n, len(g.classes_)))
    coef[g.support_] = g.dual_coef_
    for c, cls in enumerate(g.classes_):
        y = np.where(tr.labels == cls, 1, -1).astype(np.int32)
        a, r, _ = C.decomp_train_gram_dist(Kh, y, g.params)
        np.testing.assert_array_equal(coef[g.support_, c], (a * y)[g.support_])
        assert np.all(np.delete(a, g.support_) <= g.params.sv_tol)
        assert r.b == g.intercepts_b_[c] and r.iterations == g.n_iter_[c]
    assert float(np.mean(g.predict(te.compact().X) == p.predict(te.compact().X))) >= 0.995


def test_ovr_keeps_column_caches_across_classes_and_releases_them(dev, monkeypatch):
    """With the column cache on (forced at 6k) the one-vs-rest solves keep one slab per pool thread for all
    their classes and the next fit (re-allocating tens of GB per class slowed large-n solves 2-7x), with the
    same results as without the cache; release_solver_caches() hands every pool thread's slab back."""
    import ctypes

    from svm355 import OneVsRestSVC
    from svm355.models import multiclass as MC
    from svm355.models.multiclass import release_solver_caches

    tr = synthetic_mnist(6000, seed=38).compact()
    ref = OneVsRestSVC(device="cuda:0", concurrent_solves=2).fit(tr.X, tr.labels)
    monkeypatch.setenv("SVM355_DECOMP_CCACHE", "1")
    for _ in range(2):
        m = OneVsRestSVC(device="cuda:0", concurrent_solves=2).fit(tr.X, tr.labels)
        np.testing.assert_array_equal(m.dual_coef_, ref.dual_coef_)
        np.testing.assert_array_equal(m.intercepts_b_, ref.intercepts_b_)

    def slab(_):
        from svm355.ops import device as Dv

        ctx = Dv.DeviceContext.get(torch.device("cuda:0"))
        v = ctypes.c_int64(0)
        ctx.lib.svmd_cache_bytes(ctx.handle, None, ctypes.byref(v))
        return v.value

    import threading

    def per_thread(pool, workers):
        b = threading.Barrier(workers)
        return list(pool.map(lambda i: (b.wait(10), slab(i))[1], range(workers)))

    pool2 = MC._POOL[0]
    assert MC._POOL[1] == 2 and sum(per_thread(pool2, 2)) > 0  # kept for the next fit
    assert release_solver_caches()
    assert sum(per_thread(pool2, 2)) == 0
    # another width: the 2-thread pool hands its slabs back and is replaced (no pile-up across widths)
    OneVsRestSVC(device="cuda:0", concurrent_solves=2).fit(tr.X, tr.labels)
    assert sum(per_thread(pool2, 2)) > 0
    m3 = OneVsRestSVC(device="cuda:0", concurrent_solves=3).fit(tr.X, tr.labels)
    np.testing.assert_array_equal(m3.dual_coef_, ref.dual_coef_)
    assert MC._POOL[1] == 3 and MC._POOL[0] is not pool2 and pool2._shutdown
    assert sum(per_thread(MC._POOL[0], 3)) > 0 and release_solver_caches()


def test_ovr_device_model_save_load(dev, tmp_path):
    """A GPU one-vs-rest fit saved and loaded back onto the GPU (and onto the CPU) predicts the same labels;
    the coefficients, b and support ids survive the reference's text files bit for bit."""
    from svm355 import OneVsRestSVC

    tr = synthetic_mnist(2000, seed=37)
    te = synthetic_mnist(400, seed=37, offset=2000)
    X, Xt = tr.compact().X, te.compact().X
    m = OneVsRestSVC(device="cuda:0").fit(X, tr.labels)
    m.save(tmp_path / "ovr")
    g = OneVsRestSVC.load(tmp_path / "ovr", device="cuda:0")
    c = OneVsRestSVC.load(tmp_path / "ovr", device="cpu")
    for r in (g, c):
        np.testing.assert_array_equal(r.support_, m.support_)
        np.testing.assert_array_equal(r.dual_coef_, m.dual_coef_)
        np.testing.assert_array_equal(r.intercepts_b_, m.intercepts_b_)
    p = m.predict(Xt)
    np.testing.assert_array_equal(g.predict(Xt), p)
    assert float(np.mean(c.predict(Xt) == p)) >= 0.999
    np.testing.assert_allclose(g.decision_function(Xt), m.decision_function(Xt), rtol=0, atol=1e-12)


def test_gram_epilogue_exp_is_bit_identical_to_libm(dev):
    """The Gram kernel's batched exp (SGPR-sourced FMAs, igram.hip exp_batch) must equal the device
    libm exp bit for bit, so the Gram -- and every SMO trajectory -- is unchanged by it."""
    from svm355 import _native as N
    from svm355.ops.device import DeviceContext

    rng = np.random.default_rng(7)
    xs = np.concatenate([
        rng.uniform(-1.0, 0.0, 200000), rng.uniform(-40.0, 40.0, 50000), rng.uniform(-1100.0, 1100.0, 50000),
        np.array([0.0, -0.0, 1e-300, -1e-300, 5e-324, -5e-324, 1024.0, 1024.0000000000002, -1075.0,
                  -1075.0000000000002, -745.2, -708.4, 709.78, 709.79, -1e-17, np.inf, -np.inf, np.nan]),
    ])
    x = torch.from_numpy(xs).to(dev)
    lib = torch.empty_like(x)
    bat = torch.empty_like(x)
    ctx = DeviceContext.get(dev)
    N.check(ctx.lib.svmd_selftest_exp(ctx.bind(), N.ptr(x), x.numel(), N.ptr(lib), N.ptr(bat)), "svmd_selftest_exp")
    torch.cuda.synchronize()
    a = lib.cpu().numpy().view(np.uint64)
    b = bat.cpu().numpy().view(np.uint64)
    bad = np.flatnonzero(a != b)
    assert bad.size == 0, [(xs[i], lib.cpu().numpy()[i], bat.cpu().numpy()[i]) for i in bad[:5]]
