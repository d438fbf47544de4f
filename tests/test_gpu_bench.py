"""The exact commands the driver's scaling run takes, on the one GPU of the box.

* ``bench.main(["--gpus", "2", ...])`` in its default N > 1 mode -- the distributed decomposition
  solver (rehearsed with two thread ranks over the loopback transport) as the headline, then the star
  and the tree cascades (BASELINE configs 5 / 4) timed under the same bracket.
* ``torchrun --nproc-per-node 1 bench.py --gpus 1 --parallel decomp``: the per-process branch (gloo
  bootstrap, ncclCommInitRank, the RCCL candidate all-gather path, the max over ranks).
The JSON contract is checked field by field, and the timed steps against the wall clock around them."""
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

pytestmark = pytest.mark.gpu


def _check_common(out, n_gpus, steps, wall_s):
    assert out["metric"] == bench.METRIC and out["n_gpus"] == n_gpus and out["steps"] == steps
    assert out["higher_is_better"] is False and out["unit"] == "s" and out["dtype"] == "fp64"
    assert out["ms_per_step"] * steps <= wall_s * 1e3
    assert abs(out["value"] * 1e3 - out["ms_per_step"]) < 1e-3 * out["ms_per_step"] + 1e-3
    assert out["config"]["global_batch"] == 6000 and out["config"]["seq_len"] == 784


def test_bench_default_mode_two_ranks_with_the_cascades(tmp_path):
    path = tmp_path / "b.json"
    t0 = time.perf_counter()
    rc = bench.main(["--gpus", "2", "--transport", "loopback", "--steps", "1", "--warmup", "1", "--rows", "6000",
                     "--test-rows", "1000", "--baseline-1gpu", "1", "--cascade-steps", "1", "--out", str(path)])
    wall = time.perf_counter() - t0
    assert rc == 0
    out = json.loads(path.read_text())
    _check_common(out, 2, 1, wall)
    assert out["config"]["parallelism"] == "distributed-decomp-dp2-loopback"  # a one-GPU rehearsal, and labelled so
    assert out["bit_identical_to_1gpu"] is True and out["speedup_vs_1gpu"] > 0 and out["single_gpu_s"] > 0
    assert out["stop_reason"] == "converged"
    for topo in ("star", "tree"):
        c = out[f"cascade_{topo}"]
        assert out[f"cascade_{topo}_ms"] == c["ms"] > 0
        assert c["converged"] and c["rounds"] >= 1 and len(c["sv_history"]) >= 1 and c["solver"] == "per-solve"
        assert c["n_sv"] > 0 and c["accuracy"] > 0.95 and c["transport"] == "loopback"
        assert abs(c["b_minus_headline_b"]) <= 10 * 1e-5
        assert c["per_round_critical_path"] and c["critical_path_solve_ms"] > 0
    assert "merged_history" in out["cascade_star"]


def test_torchrun_one_process_default_decomp():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", "1", "--parallel", "decomp",
           "--rows", "6000", "--test-rows", "1000", "--steps", "2", "--warmup", "1", "--baseline-1gpu", "1",
           "--cascade-steps", "1"]
    t0 = time.perf_counter()
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    wall = time.perf_counter() - t0
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    _check_common(out, 1, 2, wall)
    assert out["launch"].startswith("torchrun") and out["config"]["parallelism"] == "distributed-decomp-dp1"
    assert out["launch_form"] == "one rank per process (RCCL)"
    assert out["bit_identical_to_1gpu"] is True and out["speedup_vs_1gpu"] > 0
    assert out["cascade_star"]["converged"] and out["cascade_tree"]["converged"]
    assert out["rccl_runtime"].startswith("2.")


def _torchrun(nproc, *args, env_extra=None, timeout=280):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=str(ROOT), **(env_extra or {}))
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}", "--master-addr",
           "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", str(nproc), *args]
    t0 = time.perf_counter()
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    return p, time.perf_counter() - t0


@pytest.mark.parametrize("nproc,rows", [(2, 60000), (4, 6000), (8, 60000)])
def test_torchrun_processes_share_one_gpu_over_hostcomm(nproc, rows):
    """the per-process path of the N-GPU headline (torchrun, one rank per process,
    svmd_cascade_rank_decomp) at world > 1 on the one GPU of the box.  RCCL refuses two ranks on one
    device, so the ranks exchange over the gloo group (HostCommDeviceRank: the candidate all-gather and
    the row all-gather staged through host memory); the rest -- the native driver, the block ownership,
    the replicated inner solve, bench.py's torchrun branch and timing max -- is the RCCL run's code.
    The model must equal the one-GPU decomposition solve bit for bit; at 60k the star and tree cascades
    run on the same per-process ranks too."""
    casc = "1" if rows == 60000 else "0"
    p, wall = _torchrun(nproc, "--parallel", "decomp", "--transport", "hostcomm", "--rows", str(rows),
                        "--test-rows", "1000", "--steps", "1", "--warmup", "1", "--baseline-1gpu", "1",
                        "--cascade-steps", casc)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == nproc and out["launch"].startswith("torchrun")
    assert out["config"]["parallelism"] == f"distributed-decomp-dp{nproc}-gloo" and out["config"]["global_batch"] == rows
    assert out["launch_form"].startswith("one rank per process over gloo, host-staged")
    assert out["stop_reason"] == "converged" and out["bit_identical_to_1gpu"] is True
    assert out["ms_per_step"] <= wall * 1e3
    if rows == 60000:
        assert out["n_sv"] == 1380
        for topo in ("star", "tree"):
            c = out[f"cascade_{topo}"]
            assert c["converged"] and c["transport"] == "hostcomm" and c["accuracy"] > 0.99
            assert abs(c["b_minus_headline_b"]) <= 10 * 1e-5


@pytest.mark.parametrize("nproc", [2, 4])
def test_torchrun_hostcomm_on_real_valued_rows(nproc):
    """bench.py --parallel decomp --input f64-real -- the per-process ranks on FP64
    real-valued rows (FP64-MFMA kernel values), exchanging over gloo on the one GPU: the model equals the
    one-GPU FP64 decomposition bit for bit."""
    p, wall = _torchrun(nproc, "--parallel", "decomp", "--transport", "hostcomm", "--input", "f64-real", "--rows",
                        "6000", "--test-rows", "500", "--steps", "1", "--warmup", "1", "--baseline-1gpu", "1",
                        "--cascade-steps", "0")
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["config"]["parallelism"] == f"distributed-decomp-dp{nproc}-gloo"
    assert out["host_rows"] == "fp64 (real-valued)" and out["stop_reason"] == "converged"
    assert out["bit_identical_to_1gpu"] is True and out["n_sv"] > 0


def test_torchrun_world_not_dividing_8_converges_to_the_same_model():
    """Three processes (a world that does not divide the 8-block grain): the selection's blocks are then
    a multiple of 8 x world, another trajectory to the same optimum -- the preflight checks convergence,
    b and the SV count instead of bit identity, and the line says so (bit_identity_expected false)."""
    p, wall = _torchrun(3, "--parallel", "decomp", "--transport", "hostcomm", "--rows", "6000", "--test-rows", "500",
                        "--steps", "1", "--warmup", "1", "--baseline-1gpu", "1", "--cascade-steps", "0")
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 3 and out["stop_reason"] == "converged" and out["bit_identity_expected"] is False
    assert abs(out["b_minus_1gpu_b"]) <= 1e-4 and out["fallback_reason"] is None


def test_torchrun_hostcomm_rank_failing_mid_solve_ends_every_process():
    """Rank 1 fails at outer iteration 3 of the distributed decomposition while rank 0 waits in its
    candidate all-gather: both processes exit non-zero and torchrun reports the failure, well within
    the comm deadline (the reference's MPI_Abort contract)."""
    p, wall = _torchrun(2, "--parallel", "decomp", "--transport", "hostcomm", "--rows", "6000", "--test-rows", "500",
                        "--steps", "1", "--warmup", "0", "--baseline-1gpu", "0", "--comm-timeout", "20",
                        env_extra={"SVM355_DECOMP_FAIL_RANK": "1", "SVM355_DECOMP_FAIL_OUTER": "3"}, timeout=200)
    assert p.returncode != 0
    err = p.stdout + p.stderr
    assert "injected failure of rank 1 at outer iteration 3" in err, err[-3000:]
    assert wall < 150


def test_a_failing_cascade_after_the_headline_is_reported_not_fatal():
    """The N-GPU line's cascades run after the headline was measured: a cascade rank that fails
    (SVM355_BENCH_CASCADE_FAIL) ends that cascade on every rank, the line still carries the headline and
    the error, and every process exits 0 (per-process launch, two ranks sharing the GPU)."""
    p, wall = _torchrun(2, "--parallel", "decomp", "--transport", "hostcomm", "--rows", "6000", "--test-rows", "500",
                        "--steps", "1", "--warmup", "1", "--baseline-1gpu", "0", "--cascade-steps", "1",
                        "--comm-timeout", "30", env_extra={"SVM355_BENCH_CASCADE_FAIL": "1,1"}, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["stop_reason"] == "converged" and out["value"] > 0
    assert "error" in out["cascade_star"] and "cascade_tree" not in out


def test_torchrun_refuses_to_time_gloo_under_the_rccl_label():
    """A rank whose RCCL cannot be loaded (SVM355_RCCL_LIB points nowhere): by default no timed fit runs
    over another transport -- every process exits non-zero and rank 0 names the failing rank and step
    (a SCALE run must never time gloo exchanges under an RCCL label)."""
    p, wall = _torchrun(1, "--parallel", "decomp", "--rows", "6000", "--test-rows", "500", "--steps", "1",
                        "--warmup", "1", "--baseline-1gpu", "1", "--cascade-steps", "0",
                        env_extra={"SVM355_RCCL_LIB": "/nonexistent/librccl.so"}, timeout=240)
    assert p.returncode != 0 and not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    err = p.stdout + p.stderr
    assert "the RCCL transport failed (rank 0: rank set-up" in err and "--allow-transport-fallback" in err, err[-3000:]


def test_torchrun_falls_back_to_gloo_when_allowed_and_says_so():
    """The same failure with --allow-transport-fallback: every rank falls back to the host-staged gloo
    transport before any timed fit, config.parallelism ends in -gloo, the line reports why, and the
    preflight solve equals the one-GPU solve."""
    p, wall = _torchrun(1, "--parallel", "decomp", "--rows", "6000", "--test-rows", "500", "--steps", "1",
                        "--warmup", "1", "--baseline-1gpu", "1", "--cascade-steps", "0", "--allow-transport-fallback",
                        env_extra={"SVM355_RCCL_LIB": "/nonexistent/librccl.so"}, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["config"]["parallelism"] == "distributed-decomp-dp1-gloo"
    assert out["fallback_reason"].startswith("RCCL: rank 0: rank set-up") and "gloo" in out["fallback_reason"]
    assert out["launch_form"].startswith("one rank per process over gloo")
    assert out["bit_identical_to_1gpu"] is True
