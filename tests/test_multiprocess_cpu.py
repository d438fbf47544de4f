"""The per-process cascade path (one rank per process, as the driver's torchrun launch of
``bench.py --gpus N`` runs it on N GPUs) exercised on the CPU: ``HostCommRank`` gives the native
driver gloo collectives instead of RCCL, everything else -- bench.py's torchrun branch, the
partitioning by global ids, ``fit_rank``, the solve-log gather, the timing max over ranks -- is the
code the GPUs run.  Results must be bit-identical to the same cascade on thread ranks (loopback)."""
import json
import os
import socket
import subprocess
import sys
import textwrap
import time
from pathlib import Path

import pytest

from svm355 import SVMParams
from svm355.parallel.cascade import CascadeSVM
from svm355.utils.data import synthetic_mnist

ROOT = Path(__file__).resolve().parents[1]


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=str(ROOT))
    env.pop("WORLD_SIZE", None)
    return env


def _torchrun_bench(nproc, *args, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"),
           "--gpus", str(nproc), "--device", "cpu", *args]
    p = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=timeout)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-4000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("topology,nproc", [("star", 1), ("star", 2), ("star", 3), ("tree", 4)])
def test_torchrun_ranks_match_thread_ranks(topology, nproc):
    n = 1200
    out = _torchrun_bench(nproc, "--rows", str(n), "--test-rows", "200", "--steps", "1", "--warmup", "0",
                          "--baseline-1gpu", "0", "--topology", topology, "--cascade")
    assert out["n_gpus"] == nproc and out["launch"].startswith("torchrun")
    assert out["config"]["parallelism"] == f"cascade-{topology}-dp{nproc}"
    assert out["transport"] == "hostcomm"
    # the solve log of every rank reached rank 0 (dist.all_gather_object in bench.py)
    assert out["max_rank_smo_iterations"] >= out["rank0_smo_iterations"] > 0
    assert len(out["per_round_critical_path"]) == out["rounds"]

    tr = synthetic_mnist(n, seed=2024)
    ref = CascadeSVM(SVMParams(), topology=topology).fit(tr.X, tr.y, world=nproc).result
    assert out["n_sv"] == len(ref.ids)
    assert out["b"] == ref.b  # bit-identical: same driver, same arithmetic, different transport
    assert out["rounds"] == ref.rounds and out["sv_history"] == ref.sv_history


_FAIL_SCRIPT = textwrap.dedent("""
    import datetime, sys
    import torch.distributed as dist
    from svm355 import SVMParams
    from svm355.parallel.cascade import CascadeSVM, partition_bounds
    from svm355.parallel.hostcomm import HostCommRank
    from svm355.utils.data import synthetic_mnist
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=30))
    r, P, n = dist.get_rank(), dist.get_world_size(), 800
    lo, hi = partition_bounds(n, P, r)
    tr = synthetic_mnist(hi - lo, seed=7, offset=lo)
    import numpy as np
    try:
        CascadeSVM(SVMParams(), fail_rank=1, fail_round=1).fit_rank(HostCommRank(), tr.X, tr.y, np.arange(lo, hi), n)
    except Exception as e:
        print(f"rank {r} failed: {e}", flush=True)
        sys.exit(3)
    print(f"rank {r} finished", flush=True)
""")


def test_a_failing_process_rank_ends_every_rank():
    """SURVEY §5.3 / mpi_svm_main3.cpp:420-428 (MPI_Abort): rank 1 throws at the start of round 1; rank
    0, blocked in a collective, must get an error (not hang) and both processes exit non-zero."""
    port, env = _port(), _env()
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", _FAIL_SCRIPT], cwd=ROOT, env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    t0 = time.time()
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert time.time() - t0 < 100
    assert [p.returncode for p in procs] == [3, 3], outs
    assert "rank 1 failed" in outs[1], outs[1]
    assert "rank 0 failed" in outs[0] and "hostcomm" in outs[0], outs[0]


_FAIL_ALIVE_SCRIPT = textwrap.dedent("""
    import datetime, os, sys, time
    import numpy as np
    import torch.distributed as dist
    from svm355 import SVMParams
    from svm355.parallel.cascade import CascadeSVM, partition_bounds
    from svm355.parallel.hostcomm import HostCommRank
    from svm355.utils.data import synthetic_mnist
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
    r, P, n = dist.get_rank(), dist.get_world_size(), 800
    lo, hi = partition_bounds(n, P, r)
    tr = synthetic_mnist(hi - lo, seed=7, offset=lo)
    t0 = time.time()
    try:
        CascadeSVM(SVMParams(), fail_rank=1, fail_round=1, comm_timeout_s=4.0).fit_rank(
            HostCommRank(), tr.X, tr.y, np.arange(lo, hi), n)
    except Exception as e:
        print(f"rank {r} failed after {time.time() - t0:.1f} s: {e}", flush=True)
        if r == 1:
            time.sleep(90)  # the failed rank stays alive: its socket stays open
        os._exit(3)  # MPI_Abort-like: an orderly exit would wait for the process group's teardown
    print(f"rank {r} finished", flush=True)
""")


def test_a_failing_rank_that_stays_alive_releases_its_peers():
    """The failed rank does not exit (its gloo socket stays open): its peer, blocked in a collective,
    must still leave within the fit's comm_timeout_s (4 s here), not the 300 s process-group timeout
    -- HostCommRank waits on every collective with the WaitPolicy deadline."""
    port, env = _port(), _env()
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", _FAIL_ALIVE_SCRIPT], cwd=ROOT, env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    try:
        t0 = time.time()
        out0 = procs[0].communicate(timeout=120)[0]
        elapsed = time.time() - t0
        assert procs[0].returncode == 3, out0
        assert "rank 0 failed" in out0, out0
        assert procs[1].poll() is None  # rank 1 is still alive (sleeping after its failure)
        assert elapsed < 60, (elapsed, out0)
    finally:
        procs[1].kill()
        procs[1].communicate()


def test_torchrun_cascade_cli_is_mpirun_np(tmp_path):
    """``torchrun --nproc-per-node P -m svm355 cascade`` = the reference's ``mpirun -np P`` launch
    (code/mpi_svm3.sh): every process is one rank, rank 0 prints the reference lines and writes the
    model; same model as the thread-rank CLI."""
    a, b = tmp_path / "a.json", tmp_path / "b.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "-m", "svm355", "cascade", "--cpu", "--topology", "tree",
           "--synthetic", "1000,200", "--json", str(a), "--model-dir", str(tmp_path / "m")]
    p = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    assert p.stdout.count("[rank 0] Running CascadeSVM with 2 processes") == 1  # mpi_svm_main3.cpp:430, rank 0 only
    assert "[rank 0] Cascade finished in" in p.stdout
    assert (tmp_path / "m" / "final_sv_ids.txt").exists()
    q = subprocess.run([sys.executable, "-m", "svm355", "cascade", "--cpu", "--gpus", "2", "--topology", "tree",
                        "--synthetic", "1000,200", "--json", str(b)], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=240)
    assert q.returncode == 0, q.stderr[-3000:]
    ja, jb = json.loads(a.read_text()), json.loads(b.read_text())
    assert ja["transport"] == "hostcomm" and ja["world"] == 2
    assert ja["b"] == jb["b"] and ja["n_sv"] == jb["n_sv"] and ja["rounds"] == jb["rounds"]


@pytest.mark.parametrize("nproc", [1, 2, 4])
def test_torchrun_decomp_ranks_match_one_rank(nproc):
    """The distributed decomposition solver's per-process path (bench.py --parallel decomp under torchrun,
    the launch the driver's N-GPU run takes) on its CPU twin: every process a rank over gloo
    (``HostCommRank`` -> svm_decomp_rank_train_gram), owning 1/P of the selection blocks and of f, the
    candidate records all-gathered per outer iteration.  alpha, b and the iteration counts must equal
    the one-rank solve (bench.py's bit_identical_to_1gpu compares every bit of alpha)."""
    out = _torchrun_bench(nproc, "--parallel", "decomp", "--rows", "1200", "--test-rows", "200", "--steps", "1",
                          "--warmup", "0", "--baseline-1gpu", "1")
    assert out["n_gpus"] == nproc and out["launch"].startswith("torchrun")
    assert out["config"]["parallelism"] == f"distributed-decomp-dp{nproc}"
    assert out["launch_form"] == "one rank per process (CPU oracle over gloo)"
    assert out["stop_reason"] == "converged" and out["decomp_stats"]["outer_iterations"] >= 1
    assert out["bit_identical_to_1gpu"] is True


_DECOMP_FAIL_SCRIPT = textwrap.dedent("""
    import datetime, os, sys, time
    import torch.distributed as dist
    from svm355.parallel.decomp import DistributedDecompSVC
    from svm355.parallel.hostcomm import HostCommRank
    from svm355.utils.data import synthetic_mnist
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
    r = dist.get_rank()
    tr = synthetic_mnist(1200, seed=5)
    t0 = time.time()
    try:
        DistributedDecompSVC(dist.get_world_size(), rank=HostCommRank(comm_timeout_s=8.0)).fit(tr.X, tr.y)
    except Exception as e:
        print(f"rank {r} failed after {time.time() - t0:.1f} s: {e}", flush=True)
        os._exit(3)  # MPI_Abort-like: an orderly exit would wait for the process group's teardown
    print(f"rank {r} finished", flush=True)
""")


def test_a_decomp_rank_failing_mid_solve_ends_every_process():
    """Rank 1 of 3 fails at outer iteration 2 of the distributed decomposition (SVM355_DECOMP_FAIL_RANK /
    _OUTER) while ranks 0 and 2 wait in the candidate all-gather: every process must exit non-zero
    within the deadline (the reference's MPI_Abort, mpi_svm_main3.cpp:420-428)."""
    port, env = _port(), dict(_env(), SVM355_DECOMP_FAIL_RANK="1", SVM355_DECOMP_FAIL_OUTER="2")
    procs = []
    for r in range(3):
        e = dict(env, RANK=str(r), WORLD_SIZE="3", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", _DECOMP_FAIL_SCRIPT], cwd=ROOT, env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    t0 = time.time()
    try:
        outs = [p.communicate(timeout=150)[0] for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert time.time() - t0 < 120
    assert [p.returncode for p in procs] == [3, 3, 3], outs
    assert "injected failure of rank 1 at outer iteration 2" in outs[1], outs[1]
    for r in (0, 2):
        assert f"rank {r} failed" in outs[r] and "hostcomm allgather" in outs[r], outs[r]
