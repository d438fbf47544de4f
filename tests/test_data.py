"""L0/L1: CSV reader semantics (read_CSV, main3.cpp:13-54 / gpu_svm_main4.cu:16-59), one-vs-rest
labels, min-max scaling (main3.cpp:57-89) and the synthetic MNIST-shaped generator."""
import numpy as np
import pytest

from svm355.utils.data import MinMaxScaler, compact_pixels, load_csv, one_vs_rest, synthetic_mnist, write_csv


def _write(path, text):
    path.write_text(text)
    return path


def test_csv_header_label_mapping(tmp_path):
    p = _write(tmp_path / "a.csv", "x0,x1,label\n1,2,1\n3.5,-4,7\n0,0,1\n")
    ds = load_csv(p)
    assert ds.n == 3 and ds.d == 2
    np.testing.assert_array_equal(ds.X, [[1, 2], [3.5, -4], [0, 0]])
    np.testing.assert_array_equal(ds.y, [1, -1, 1])
    np.testing.assert_array_equal(ds.labels, [1, 7, 1])


def test_csv_positive_label_and_crlf(tmp_path):
    p = _write(tmp_path / "b.csv", "a,b,y\r\n1,2,3\r\n4,5,1\r\n")
    ds = load_csv(p, positive_label=3)
    np.testing.assert_array_equal(ds.y, [1, -1])


def test_csv_short_lines_skipped_and_counted_by_limit(tmp_path):
    # Lines with < 2 fields are skipped; the gpu_svm4 limit counts them (gpu_svm_main4.cu:34-38).
    p = _write(tmp_path / "c.csv", "a,b,y\n1,2,1\n\n3,4,0\n5,6,1\n")
    assert load_csv(p).n == 3
    assert load_csv(p, limit=2).n == 1  # line 2 is empty: consumed by the limit, not kept
    assert load_csv(p, limit=3).n == 2


def test_csv_errors(tmp_path):
    with pytest.raises(FileNotFoundError):
        load_csv(tmp_path / "missing.csv")
    p = _write(tmp_path / "bad.csv", "a,b,y\n1,2\n")  # wrong width
    with pytest.raises(FileNotFoundError, match="malformed"):
        load_csv(p)


def test_csv_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    X = rng.normal(size=(17, 5))
    X[:, 0] = rng.integers(0, 256, 17)
    lab = rng.integers(0, 10, 17).astype(np.int32)
    write_csv(tmp_path / "r.csv", X, lab)
    ds = load_csv(tmp_path / "r.csv")
    np.testing.assert_array_equal(ds.X, X)  # %.17g round-trips exactly
    np.testing.assert_array_equal(ds.labels, lab)


def test_one_vs_rest():
    np.testing.assert_array_equal(one_vs_rest([0, 1, 2, 1]), [-1, 1, -1, 1])


def test_scaler_matches_reference_formula():
    rng = np.random.default_rng(1)
    X = rng.integers(0, 256, size=(50, 6)).astype(float)
    X[:, 2] = 7.0  # constant column: range < 1e-12 -> 1
    s = MinMaxScaler().fit(X)
    np.testing.assert_array_equal(s.min_, X.min(0))
    np.testing.assert_array_equal(s.max_, X.max(0))
    rng_ = X.max(0) - X.min(0)
    rng_[rng_ < 1e-12] = 1.0
    np.testing.assert_array_equal(s.transform(X), (X - X.min(0)) / rng_)
    assert np.all(s.transform(X)[:, 2] == 0.0)


def test_synthetic_mnist_shape_and_determinism():
    a = synthetic_mnist(300, seed=3)
    b = synthetic_mnist(100, seed=3, offset=200)
    assert a.X.shape == (300, 784)
    np.testing.assert_array_equal(a.X[200:], b.X)
    np.testing.assert_array_equal(a.labels[200:], b.labels)
    assert np.all(a.X == np.round(a.X)) and a.X.min() >= 0 and a.X.max() <= 255
    assert set(np.unique(a.labels)) <= set(range(10))
    frac_pos = np.mean(a.y == 1)
    assert 0.05 < frac_pos < 0.2  # digit "1" ~ 11%
    assert 0.1 < np.mean(a.X > 0) < 0.35  # MNIST-like sparsity (~19% ink)
    c = synthetic_mnist(300, seed=4)
    assert not np.array_equal(a.X, c.X)


def test_compact_pixels_exact_bytes_only():
    a = synthetic_mnist(50, seed=5)
    c = a.compact()
    assert c.X.dtype == np.uint8 and np.array_equal(c.X.astype(np.float64), a.X)
    assert c.y is a.y and compact_pixels(c.X) is c.X
    for bad in (np.array([[0.5, 1.0]]), np.array([[256.0]]), np.array([[-1.0]]), np.array([[np.nan]])):
        assert compact_pixels(bad) is None
    assert c.compact() is c and (c.n, c.d) == (a.n, a.d)
