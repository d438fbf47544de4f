"""Native Cascade SVM (bin/svm_cascade: one process, a thread per rank, RCCL or loopback transport)
against the Python driver on the same device solver: same rounds, same SV ids, the same b bit for bit.

RCCL refuses two ranks on one GPU, so multi-rank runs here use the loopback transport (exchanges
staged through host memory); the RCCL transport is exercised with one rank."""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

from svm355 import SVMParams
from svm355.parallel.cascade import CascadeSVM, partition_bounds
from svm355.parallel.transport import run_threads
from svm355.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu

EXE = Path(__file__).resolve().parents[1] / "svm355" / "bin" / "svm_cascade"
N, M = 2000, 500


def _native(tmp_path, topology, world, transport):
    out = tmp_path / f"{topology}{world}{transport}.json"
    r = subprocess.run([str(EXE), "--synthetic", f"{N},{M}", "--topology", topology, "--gpus", str(world),
                        "--transport", transport, "--json", str(out), "--quiet"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(out.read_text()), r.stdout


def _python(topology, world):
    tr = synthetic_mnist(N, seed=2024)
    te = synthetic_mnist(M, seed=2024, offset=N)
    dev = torch.device("cuda:0")

    def fn(t):
        lo, hi = partition_bounds(N, t.world, t.rank)
        c = CascadeSVM(t, SVMParams(), topology=topology, verbose=0, device=dev)
        c.fit(tr.X[lo:hi], tr.y[lo:hi], np.arange(lo, hi), n_total=N)
        return c.summary(), sorted(c.result.sv.ids.tolist()), int((c.predict(te.X) == te.y).sum())

    return run_threads(world, fn, device_for_rank=lambda r: dev)[0]


@pytest.mark.parametrize("topology,world", [("star", 1), ("star", 2), ("star", 3), ("tree", 2), ("tree", 4)])
def test_native_loopback_cascade_matches_python_driver(tmp_path, topology, world):
    nat, stdout = _native(tmp_path, topology, world, "loopback")
    summ, ids, correct = _python(topology, world)
    assert nat["converged"] and summ["converged"]
    assert nat["rounds"] == summ["rounds"]
    assert nat["sv_history"] == summ["sv_history"]
    assert nat["sv_ids"] == ids
    assert nat["b"] == summ["b"]  # same solver, same merge order: bit-identical
    assert nat["test_correct"] == correct
    # the reference's stdout contract
    head = "modified CascadeSVM" if topology == "star" else "CascadeSVM"
    assert f"[rank 0] Running {head} with {world} processes" in stdout
    assert f"[rank 0] total samples = {N}, features = 784" in stdout
    assert "[rank 0] Final b = " in stdout and f"[rank 0] Cascade finished in {nat['rounds']} rounds" in stdout


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_native_rccl_single_rank_equals_loopback(tmp_path, topology):
    rc, _ = _native(tmp_path, topology, 1, "rccl")
    lb, _ = _native(tmp_path, topology, 1, "loopback")
    assert rc["transport"] == "rccl" and lb["transport"] == "loopback"
    assert rc["sv_ids"] == lb["sv_ids"] and rc["b"] == lb["b"] and rc["rounds"] == lb["rounds"]


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_native_checkpoint_resume_matches_uninterrupted_run(tmp_path, topology):
    """Stop after 2 rounds with a checkpoint, resume from it: the same rounds, SV ids and b, bit for
    bit, as one uninterrupted run (the carried state is exactly the global SV set and b)."""
    full, _ = _native(tmp_path, topology, 2, "loopback")
    ck = tmp_path / f"ck_{topology}"

    def run(extra, name):
        out = tmp_path / name
        r = subprocess.run([str(EXE), "--synthetic", f"{N},{M}", "--topology", topology, "--gpus", "2",
                            "--transport", "loopback", "--json", str(out), "--quiet", *extra],
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stdout + r.stderr
        return json.loads(out.read_text()), r.stdout

    part, _ = run(["--max-rounds", "2", "--checkpoint-dir", str(ck)], "part.json")
    assert part["rounds"] == 2 and not part["converged"] and (ck / "cascade_state.bin").exists()
    res, stdout = run(["--checkpoint-dir", str(ck), "--resume"], "resumed.json")
    assert "[rank 0] resumed from checkpoint at round 2" in stdout
    assert res["converged"] and res["rounds"] == full["rounds"]
    assert res["sv_ids"] == full["sv_ids"] and res["b"] == full["b"]
    assert res["test_correct"] == full["test_correct"]
