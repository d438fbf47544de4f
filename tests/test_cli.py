"""CLI entry points (python -m svm355 ...): reference stdout contract and JSON summaries (CPU)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(args, tmp_path, timeout=600):
    env = dict(os.environ, MASTER_PORT=str(29600 + os.getpid() % 300))
    r = subprocess.run([sys.executable, "-m", "svm355", *args], cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_cli_help(tmp_path):
    out = _run(["--help"], tmp_path)
    assert "serial" in out and "cascade" in out


def test_cli_serial_reference_lines(tmp_path):
    js = tmp_path / "s.json"
    out = _run(["serial", "--synthetic", "600,200", "--json", str(js), "--model-dir", str(tmp_path / "m")], tmp_path)
    lines = [l.split("=")[0].split(":")[0].strip() for l in out.strip().splitlines()]
    assert lines == ["n", "n_features", "number of iterations", "b", "(b_high - b_low)/2*1e10", "Final SV count",
                     "Test accuracy", "Training time", "Prediction time", "Total Runtime"]
    s = json.loads(js.read_text())
    assert s["stop_reason"] == "converged" and s["n"] == 600
    for f in ("final_sv_ids.txt", "final_sv_labels.txt", "final_sv_alphas.txt", "final_b.txt"):
        assert (tmp_path / "m" / f).exists()


def test_cli_serial_second_order_selection(tmp_path):
    """--wss second: the opt-in second-order selection reaches the same model in fewer iterations."""
    runs = {}
    for wss in ("first", "second"):
        js = tmp_path / f"{wss}.json"
        _run(["serial", "--synthetic", "600,200", "--wss", wss, "--json", str(js)], tmp_path)
        runs[wss] = json.loads(js.read_text())
    f, s = runs["first"], runs["second"]
    assert s["stop_reason"] == f["stop_reason"] == "converged"
    assert s["iterations"] < f["iterations"]
    assert s["n_sv"] == f["n_sv"] and s["accuracy"] == f["accuracy"]


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_cli_cascade_single_rank_cpu(tmp_path, topology):
    js = tmp_path / "c.json"
    out = _run(["cascade", "--synthetic", "700,200", "--cpu", "--topology", topology, "--json", str(js)], tmp_path)
    assert "[rank 0] Running" in out and "[rank 0] Final b = " in out
    assert "[rank 0] Cascade finished in" in out and "[rank 0] training time =" in out
    s = json.loads(js.read_text())
    assert s["converged"] and s["world"] == 1 and s["accuracy"] > 0.9


def test_cli_cascade_two_ranks_cpu(tmp_path):
    js = tmp_path / "c2.json"
    out = _run(["cascade", "--synthetic", "900,200", "--cpu", "--gpus", "2", "--json", str(js),
                "--model-dir", str(tmp_path / "m")], tmp_path, timeout=900)
    assert "[rank 0] Running modified CascadeSVM with 2 processes" in out
    assert "[rank 0] merged unique SV count from workers = " in out and "=== Round 0 ===" in out
    s = json.loads(js.read_text())
    assert s["converged"] and s["world"] == 2 and s["backend"] == "cpu"
    assert {x["rank"] for x in s["solves"]} == {0, 1}
    for f in ("final_sv_ids.txt", "final_sv_labels.txt", "final_sv_alphas.txt", "final_b.txt"):
        assert (tmp_path / "m" / f).exists()


def test_native_cascade_rejects_non_power_of_two_tree():
    """bin/svm_cascade aborts a classical cascade on a non-power-of-2 world (mpi_svm_main3.cpp:420-428)
    before touching a GPU, so this runs on a CPU-only host too."""
    exe = Path(__file__).resolve().parents[1] / "svm355" / "bin" / "svm_cascade"
    r = subprocess.run([str(exe), "--topology", "tree", "--gpus", "3", "--synthetic", "100,10"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    assert "power-of-2" in r.stderr


def test_cli_multiclass_two_ranks_gloo(tmp_path):
    js = tmp_path / "mc.json"
    out = _run(["multiclass", "--synthetic", "500,200", "--cpu", "--gpus", "2", "--backend", "gloo",
                "--json", str(js), "--model-dir", str(tmp_path / "model")], tmp_path, timeout=600)
    assert "[rank 0] one-vs-rest over 10 classes on 2 rank(s)" in out
    s = json.loads(js.read_text())
    assert s["world"] == 2 and all(r == "converged" for r in s["stop_reasons"]) and s["accuracy"] > 0.8
    from svm355 import OneVsRestSVC

    m = OneVsRestSVC.load(tmp_path / "model")  # the distributed fit's model, saved by rank 0
    assert len(m.classes_) == 10 and (tmp_path / "model" / "class_1" / "final_b.txt").exists()


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_cli_scale_sweeps_rank_counts(tmp_path, topology):
    """scale = mpi_svm2.sh / mpi_svm3.sh over P: one row per rank count (the tree skips P = 3), the
    single-device baseline, and the same converged model at every P (CPU thread-ranks)."""
    js = tmp_path / "scale.json"
    out = _run(["scale", "--cpu", "--trainer", "cascade", "--synthetic", "500,200", "--ranks", "1,2,3,4",
                "--topology", topology, "--repeats", "1", "--warmup", "0", "--json", str(js)], tmp_path)
    s = json.loads(js.read_text())
    assert s["device"] == "cpu" and len(s["sizes"]) == 1 and s["sizes"][0]["n"] == 500
    sz = s["sizes"][0]
    assert sz["single_n_sv"] > 0
    rows = sz["rows"]
    assert [r["P"] for r in rows] == ([1, 2, 3, 4] if topology == "star" else [1, 2, 4])
    for r in rows:
        assert r["converged"] and r["rounds"] >= 1 and r["n_sv"] > 0
        assert r["accuracy"] > 0.9
        assert r["critical_path_solve_ms"] > 0 and r["efficiency_vs_single"] > 0
    assert "efficiency" in out and "single CPU oracle" in out


def test_cli_scale_max_iter_caps_every_solve(tmp_path):
    """--max-iter reaches the single-device baseline and the cascade's solves (large n needs more than
    the reference's 100,000)."""
    js = tmp_path / "scale.json"
    _run(["scale", "--cpu", "--trainer", "cascade", "--synthetic", "500,100", "--ranks", "1", "--repeats", "1",
          "--warmup", "0", "--max-iter", "7", "--json", str(js)], tmp_path)
    sz = json.loads(js.read_text())["sizes"][0]
    assert sz["single_iterations"] <= 8  # the oracle counts the iteration that finds the cap reached


def test_cli_scale_decomp_needs_a_gpu(tmp_path):
    """The default trainer is the distributed decomposition, which runs on GPUs: --cpu asks for the cascade."""
    r = subprocess.run([sys.executable, "-m", "svm355", "scale", "--cpu", "--synthetic", "400,100"], cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "--trainer cascade" in r.stderr


def test_cli_configuration_errors_exit_2_without_a_traceback(tmp_path):
    """A bad configuration (the tree cascade on 3 ranks; the reference MPI_Aborts, mpi_svm_main3.cpp:420-428)
    ends the CLI with exit status 2 and one line naming the problem."""
    r = subprocess.run([sys.executable, "-m", "svm355", "cascade", "--synthetic", "600,100", "--cpu", "--gpus", "3",
                        "--topology", "tree"], cwd=tmp_path, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=str(ROOT)))
    assert r.returncode == 2 and "power-of-2" in r.stderr and "Traceback" not in r.stderr, r.stderr[-2000:]
