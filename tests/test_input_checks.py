"""Input validation of the distributed entry points (CPU: the checks run before any device work).

SVC.fit rejects labels other than +1/-1 and non-(n, d) shapes (models/svc.py); the distributed
solvers must too -- a 0 label falls in neither I_high nor I_low (main3.cpp:107-142), so a solve would
'converge' to a wrong model -- and the integer-row solvers must refuse non-pixel values instead of
casting them (3.7 -> 3, 300 -> 44)."""
import datetime

import numpy as np
import pytest

from svm355.parallel.decomp import _fit_native, _rows
from svm355.parallel.dsmo import DsmoGroup, DsmoRank
from svm355.utils.config import SVMParams
from svm355.utils.data import check_labels, pixel_rows


def _data(n=8, d=4):
    rng = np.random.default_rng(0)
    return rng.integers(0, 256, size=(n, d)).astype(np.uint8), np.where(np.arange(n) % 2 == 0, 1, -1)


def test_check_labels_and_pixel_rows():
    X, y = _data()
    assert check_labels(y, 8).dtype == np.int32
    with pytest.raises(ValueError, match=r"\+1/-1"):
        check_labels(np.where(y > 0, 1, 0), 8)
    with pytest.raises(ValueError, match="shape"):
        check_labels(y[:5], 8)
    assert pixel_rows(X.astype(np.float64), "x").dtype == np.uint8
    for bad in (X.astype(np.float64) + 0.5, X.astype(np.float64) * 2, -X.astype(np.float64) - 1):
        with pytest.raises(ValueError, match="integer pixel rows"):
            pixel_rows(bad, "x")


def _never(*a):  # the native solve must not be reached
    raise AssertionError("native entry point called with invalid input")


@pytest.mark.parametrize("bad", ["labels01", "shape", "real_rows", "wrapped_rows"])
def test_distributed_entry_points_reject_bad_input(bad):
    X, y = _data()
    if bad == "labels01":
        y = np.where(y > 0, 1, 0)
    elif bad == "shape":
        y = y[:5]
    elif bad == "real_rows":
        X = X.astype(np.float64) + 0.25
    else:
        X = X.astype(np.float64) + 200.0  # values above 255 would wrap in a uint8 cast
    if bad in ("labels01", "shape"):
        with pytest.raises(ValueError):
            _fit_native(_never, None, X, y, SVMParams(), 1024, 1)
    else:  # the decomposition entry points train non-pixel rows as FP64 rows -- never a uint8 cast
        rows, u8 = _rows(X)
        assert not u8 and rows.dtype == np.float64 and np.array_equal(rows, X)
    with pytest.raises(ValueError):  # the pairwise solvers take pixel rows only
        DsmoGroup.fit(object.__new__(DsmoGroup), X, y)


def test_dsmo_rank_agrees_on_a_bad_input_before_any_solve():
    """The per-process form validates inside its collective protocol: every rank learns of the failure
    from the first all-reduce and raises (one gloo rank here)."""
    import torch.distributed as dist

    store = dist.HashStore()
    dist.init_process_group("gloo", store=store, rank=0, world_size=1, timeout=datetime.timedelta(seconds=30))
    try:
        X, y = _data()
        r = object.__new__(DsmoRank)
        r.handle = None
        with pytest.raises(ValueError, match="failed on some rank"):
            DsmoRank.fit(r, X, np.where(y > 0, 1, 0))
        with pytest.raises(ValueError, match="failed on some rank"):
            DsmoRank.fit(r, X.astype(np.float64) + 0.5, y)
    finally:
        dist.destroy_process_group()



@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf])
def test_non_finite_rows_are_rejected_on_the_cpu(bad):
    """A NaN or an infinity in X: a clear error, not an empty model (the column bounds propagate NaN)."""
    from svm355 import SVC, OneVsRestSVC

    rng = np.random.default_rng(2)
    X = rng.random((120, 6))
    X[37, 4] = bad
    y = np.where(rng.random(120) < 0.5, 1, -1).astype(np.int32)
    with pytest.raises(ValueError, match="NaN or infinite"):
        SVC(device="cpu").fit(X, y)
    with pytest.raises(ValueError, match="NaN or infinite"):
        SVC(device="cpu", scale=False).fit(X, y)
    with pytest.raises(ValueError, match="NaN or infinite"):
        OneVsRestSVC(device="cpu").fit(X, rng.integers(0, 3, size=120))


def test_non_finite_csv_cell_is_a_malformed_line(tmp_path):
    from svm355.utils.data import load_csv

    p = tmp_path / "d.csv"
    p.write_text("f0,f1,label\n0.5,1.0,1\n0.25,nan,0\n")
    with pytest.raises(FileNotFoundError, match="malformed CSV line 3"):  # load_csv's error type (test_data.py)
        load_csv(p)


def test_prediction_rows_must_have_the_training_width():
    from svm355 import SVC, OneVsRestSVC

    rng = np.random.default_rng(4)
    X = rng.random((150, 5))
    y = np.where(rng.random(150) < 0.5, 1, -1).astype(np.int32)
    for m in (SVC(device="cpu").fit(X, y), OneVsRestSVC(device="cpu", n_threads=2).fit(X, rng.integers(0, 3, 150))):
        with pytest.raises(ValueError, match=r"\(m, 5\)"):
            m.predict(rng.random((10, 4)))
        with pytest.raises(ValueError, match=r"\(m, 5\)"):
            m.decision_function(rng.random(5))
        assert m.predict(np.empty((0, 5))).shape == (0,)


@pytest.mark.parametrize("kw", [dict(C=0.0), dict(C=-1.0), dict(gamma=0.0), dict(tau=0.0), dict(max_iter=0),
                                dict(eps=-1e-12), dict(C=float("nan")), dict(wss=3)])
def test_parameters_out_of_range_are_rejected(kw):
    from svm355 import SVC

    with pytest.raises(ValueError, match="out of range"):
        SVMParams(**kw)
    key = {"tau": "tol"}.get(next(iter(kw)), next(iter(kw)))
    if key != "wss":
        with pytest.raises(ValueError, match="out of range"):
            SVC(**{key: kw[next(iter(kw))]})


def test_native_cli_rejects_parameters_out_of_range(tmp_path):
    import subprocess
    from pathlib import Path

    exe = Path(__file__).resolve().parents[1] / "svm355" / "bin" / "svm_serial"
    for args in (["--C", "-1"], ["--gamma", "0"], ["--max-iter", "0"]):
        r = subprocess.run([str(exe), "--synthetic", "20,5", *args], cwd=tmp_path, capture_output=True, text=True,
                           timeout=60)
        assert r.returncode == 2 and "out of range" in r.stderr, (args, r.stdout, r.stderr)
    # values parse whole: no silent 0 from atoll("abc") (which read the default CSVs) or 1e-5 from "1e-5x"
    bad = ((["--synthetic", "abc"], "invalid integer"), (["--synthetic", "20,x"], "invalid integer"),
           (["--synthetic", "0,5"], "N >= 1"), (["--synthetic", "20,5", "--C", "1e-5x"], "invalid number"),
           (["--synthetic", "20,5", "--n-limit", "10,5"], "invalid integer"),
           (["--synthetic", "20,5", "--gram", "bogus"], "--gram must be"))
    for args, msg in bad:
        r = subprocess.run([str(exe), *args], cwd=tmp_path, capture_output=True, text=True, timeout=60)
        assert r.returncode == 2 and msg in r.stderr, (args, r.stdout, r.stderr)
    casc = exe.parent / "svm_cascade"
    for args in (["--gpus", "two"], ["--max-rounds", "0"], ["--comm-timeout", "0"]):
        r = subprocess.run([str(casc), "--synthetic", "40,10", *args], cwd=tmp_path, capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 2, (args, r.stdout, r.stderr)


def test_warm_starts_must_be_feasible():
    """SVC.fit(alpha0=...) and the oracles' alpha: the right length (the native solvers read n entries),
    finite, inside [0, C] and on sum(alpha y) = 0 -- from an infeasible start a solver stops on a
    'converged' model that is not a solution."""
    from svm355 import SVC
    from svm355.ops import cpu as C

    rng = np.random.default_rng(6)
    X = rng.random((100, 4))
    y = np.where(rng.random(100) < 0.5, 1, -1).astype(np.int32)
    for a0, msg in ((np.zeros(10), "shape"), (np.full(100, 20.0), r"\[0, C"), (-np.ones(100), r"\[0, C"),
                    (np.where(y > 0, 1.0, 0.0), "sum"), (np.full(100, np.nan), r"\[0, C")):
        with pytest.raises(ValueError, match=msg):
            SVC(device="cpu").fit(X, y, alpha0=a0)
    K = C.rbf_matrix(X, X, 0.5)
    with pytest.raises(ValueError, match="shape"):
        C.smo_train_gram(K, y, SVMParams(gamma=0.5), alpha=np.zeros(10), warm=True)
    with pytest.raises(ValueError, match="at least"):
        C.decomp_train_gram(K[:50, :50], y, SVMParams(gamma=0.5))
    feasible = np.zeros(100)
    i, j = int(np.flatnonzero(y > 0)[0]), int(np.flatnonzero(y < 0)[0])
    feasible[i] = feasible[j] = 0.5
    assert SVC(device="cpu").fit(X, y, alpha0=feasible).stop_reason_ == "converged"
    # a solver's own solution sits a few ulps outside the box (a_i moves by the rounded step of a_j): it
    # stays a valid warm start
    m = SVC(device="cpu", C=1.0, gamma=0.5).fit(X, y)
    a = m.alpha_.copy()
    a[np.argmax(a)] = 1.0 + 2e-15
    a[np.argmin(a)] = -1e-15
    assert SVC(device="cpu", C=1.0, gamma=0.5).fit(X, y, alpha0=a).stop_reason_ == "converged"
