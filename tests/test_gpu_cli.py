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
