"""SVC estimator on the CPU backend, model files (mpi_svm_main3.cpp:754-770 format) and the serial CLI."""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

import svm355
from svm355.ops import cpu as C
from svm355.utils.data import MinMaxScaler, write_csv

ROOT = Path(__file__).resolve().parents[1]


def test_svc_cpu_fit_predict(small_mnist):
    tr, te = small_mnist
    m = svm355.SVC(device="cpu", n_threads=4).fit(tr.X, tr.y)
    assert m.stop_reason_ == "converged"
    assert 0 < len(m.support_) < tr.n
    assert m.score(te.X, te.y) > 0.95
    # same numbers as the raw oracle on pre-scaled data
    a, res, _ = C.smo_train(MinMaxScaler().fit_transform(tr.X), tr.y, m.params)
    np.testing.assert_array_equal(a, m.alpha_)
    assert res.b == m.b_
    np.testing.assert_array_equal(m.dual_coef_, a[m.support_] * tr.y[m.support_])


def test_predict_zero_rule():
    m = svm355.SVC(device="cpu")
    m.decision_function = lambda X: np.array([0.0, 1.0, -1.0])
    assert m.predict(None).tolist() == [-1, 1, -1]  # main3.cpp:400: curr > 0 ? 1 : -1
    m.zero_is_positive = True
    assert m.predict(None).tolist() == [1, 1, -1]  # cascade: s >= 0 ? 1 : -1


def test_model_files_roundtrip(tmp_path, small_mnist):
    tr, te = small_mnist
    m = svm355.SVC(device="cpu", n_threads=4).fit(tr.X, tr.y)
    m.save(tmp_path / "model")
    for name in ("final_sv_ids.txt", "final_sv_labels.txt", "final_sv_alphas.txt", "final_b.txt"):
        assert (tmp_path / "model" / name).exists()
    ids = np.loadtxt(tmp_path / "model" / "final_sv_ids.txt", dtype=np.int64)
    np.testing.assert_array_equal(ids, m.support_)
    alphas = np.loadtxt(tmp_path / "model" / "final_sv_alphas.txt")
    np.testing.assert_array_equal(alphas, m.alpha_[m.support_])  # %.17g is exact
    m2 = svm355.SVC.load(tmp_path / "model", device="cpu")
    assert m2.b_ == m.b_
    np.testing.assert_array_equal(m2.decision_function(te.X), m.decision_function(te.X))


def test_serial_cli_output_contract(tmp_path, small_mnist):
    tr, te = small_mnist
    write_csv(tmp_path / "toy_train_data.csv", tr.X[:400], tr.labels[:400])
    write_csv(tmp_path / "toy_test_data.csv", te.X[:100], te.labels[:100])
    exe = ROOT / "svm355" / "bin" / "svm_serial"
    if not exe.exists():
        pytest.skip("native CLIs not built")
    out = subprocess.run([str(exe), "--dataset", "toy", "--json", "s.json", "--model-dir", "mdl"], cwd=tmp_path,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().splitlines()
    heads = ["n = 400", "n_features = 784", "number of iterations: ", "b = ", "(b_high - b_low)/2*1e10 = ",
             "Final SV count = ", "Test accuracy = ", "Training time: ", "Prediction time: ", "Total Runtime: "]
    assert len(lines) == len(heads)
    for line, h in zip(lines, heads):
        assert line.startswith(h), (line, h)
    js = json.loads((tmp_path / "s.json").read_text())
    m = svm355.SVC(device="cpu", n_threads=4).fit(tr.X[:400], tr.y[:400])
    assert js["iterations"] == m.n_iter_ and js["b"] == m.b_ and js["n_sv"] == len(m.support_)
    assert (tmp_path / "mdl" / "final_b.txt").exists()
