"""The single-GPU CLI (``python -m svm355 gpu``: gpu_svm_main3.cu) and the size sweep (``sweep``:
gpu_svm4.sh) on the GPU, with the reference's pairwise SMO and with ``--solver decomp``."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _run(args, timeout=300):
    r = subprocess.run([sys.executable, "-m", "svm355", *args], cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout, env=dict(os.environ))
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def _field(out, name):
    line = next(l for l in out.splitlines() if l.startswith(name))
    return line.split("=", 1)[1].strip() if "=" in line else line.split(":", 1)[1].strip()


def test_gpu_cli_pairwise_and_decomposition_agree(tmp_path):
    runs = {}
    for solver in ("smo", "decomp"):
        js = tmp_path / f"{solver}.json"
        out = _run(["gpu", "--synthetic", "6000,2000", "--solver", solver, "--json", str(js), "--quiet"])
        lines = [l.split("=")[0].split(":")[0].strip() for l in out.strip().splitlines()]
        assert lines == ["n", "n_features", "number of iterations", "b", "(b_high - b_low)/2*1e10",
                         "Test accuracy", "Final SV count", "The training time", "The prediction time",
                         "The elapsed time"], out
        runs[solver] = (json.loads(js.read_text()), int(_field(out, "Final SV count")))
    (smo, nsv_smo), (dec, nsv_dec) = runs["smo"], runs["decomp"]
    assert smo["solver"] == "smo" and dec["solver"] == "decomp"
    assert smo["stop_reason"] == dec["stop_reason"] == "converged"
    # the same optimality test on all n points: the same support vectors, b within 10 tau
    assert nsv_dec == nsv_smo > 0
    assert abs(dec["b"] - smo["b"]) <= 10 * smo["tau"]
    assert dec["accuracy"] == pytest.approx(smo["accuracy"], abs=2e-3)


def test_gpu_sweep_with_the_decomposition_solver(tmp_path):
    js = tmp_path / "sweep.json"
    out = _run(["sweep", "--sizes", "3000,6000", "--out", str(js), "--synthetic", "6000,1000", "--solver", "decomp"])
    rows = json.loads(js.read_text())
    assert [r["n"] for r in rows] == [3000, 6000]
    assert all(r["solver"] == "decomp" and r["stop_reason"] == "converged" for r in rows)
    assert "n train" in out


EXE = ROOT / "svm355" / "bin" / "svm_gpu"


def test_native_svm_gpu_on_reference_csv_files(tmp_path):
    """bin/svm_gpu (gpu_svm_main3.cu's program) on CSV files in the reference's format: its stdout lines in
    the reference's order, the reference's four model files, and the same SV count with the default
    (decomposition) and the pairwise (--solver smo) solver."""
    from svm355.utils.data import synthetic_mnist, write_csv

    tr, te = synthetic_mnist(5000, seed=61), synthetic_mnist(1000, seed=61, offset=5000)
    write_csv(tmp_path / "mnist3_train_data.csv", tr.X, tr.labels)
    write_csv(tmp_path / "mnist3_test_data.csv", te.X, te.labels)
    nsv = {}
    for solver in ("auto", "smo"):
        md = tmp_path / f"model_{solver}"
        r = subprocess.run([str(EXE), "--solver", solver, "--model-dir", str(md), "--json", str(tmp_path / f"{solver}.json")],
                           cwd=tmp_path, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        lines = [l.split("=")[0].split(":")[0].strip() for l in r.stdout.strip().splitlines()]
        assert lines == ["n", "n_features", "number of iterations", "b", "(b_high - b_low)/2*1e10",
                         "Test accuracy", "Final SV count", "The training time", "The prediction time",
                         "The elapsed time"], r.stdout
        assert _field(r.stdout, "n") == "5000" and _field(r.stdout, "n_features") == "784"
        for f in ("final_sv_ids.txt", "final_sv_labels.txt", "final_sv_alphas.txt", "final_b.txt"):
            assert (md / f).exists()
        nsv[solver] = int(_field(r.stdout, "Final SV count"))
        js = json.loads((tmp_path / f"{solver}.json").read_text())
        assert js["stop_reason"] == "converged" and js["accuracy"] > 0.98
    assert nsv["auto"] == nsv["smo"] > 0


def test_multiclass_cli_on_the_gpu(tmp_path):
    """python -m svm355 multiclass on the GPU (the decomposition solver per class by default, the batched
    pairwise launch with --solver batched): every class converged, the same predictions' accuracy, and a
    saved model that loads back."""
    acc = {}
    for solver in ("auto", "batched"):
        js = tmp_path / f"{solver}.json"
        out = _run(["multiclass", "--synthetic", "6000,1000", "--solver", solver, "--json", str(js),
                    "--model-dir", str(tmp_path / f"m_{solver}")])
        s = json.loads(js.read_text())
        assert "[rank 0] one-vs-rest over 10 classes on 1 rank(s)" in out
        assert all(r == "converged" for r in s["stop_reasons"])
        assert s["solver"] == ("decomp" if solver == "auto" else "batched")
        acc[solver] = s["accuracy"]
    assert abs(acc["auto"] - acc["batched"]) <= 2e-3
    from svm355 import OneVsRestSVC

    assert len(OneVsRestSVC.load(tmp_path / "m_auto").classes_) == 10
