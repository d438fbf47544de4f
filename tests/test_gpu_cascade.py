"""Cascade SVM on the gfx950 backend (csrc/hip/cascade_dev.hip) driven by the one native driver.

* HIP backend vs the CPU-oracle backend on the same partitions (kernel values differ in the last
  ulps between the MFMA norm form and the direct sum, so tolerances);
* RCCL transport (group of one GPU, and a per-process rank bootstrapped from an ncclUniqueId) vs
  the loopback transport: bit-identical;
* the native CLI bin/svm_cascade: reference stdout lines, checkpoint/resume, fault injection.

RCCL refuses two ranks on one GPU, so multi-rank runs on the one-GPU box use the loopback
transport; RCCL itself runs here with one rank (ncclCommInitAll and ncclCommInitRank)."""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

from svm355 import SVC, SVMParams
from svm355._native import NativeError
from svm355.parallel.cascade import CascadeSVM, preflight_script
from svm355.parallel.rccl import DeviceGroup, RcclRank, rccl_info
from svm355.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu

EXE = Path(__file__).resolve().parents[1] / "svm355" / "bin" / "svm_cascade"
N, M = 2000, 500


@pytest.fixture(scope="module")
def data():
    return synthetic_mnist(N, seed=21), synthetic_mnist(M, seed=21, offset=N)


@pytest.mark.parametrize("solver", ["smo", "decomp"])
@pytest.mark.parametrize("topology,world", [("star", 1), ("star", 2), ("star", 3), ("tree", 2), ("tree", 4)])
def test_hip_cascade_matches_cpu_cascade(data, topology, world, solver):
    """The device cascade against the CPU oracle's, with either solver for every local / merge solve
    (decomp: the warm-started decomposition on the device, its CPU oracle on the direct-RBF Gram)."""
    tr, te = data
    g = CascadeSVM(SVMParams(), topology=topology, solver=solver).fit(tr.compact().X, tr.y, world=world,
                                                                      device="cuda", transport="loopback")
    c = CascadeSVM(SVMParams(n_threads=4), topology=topology, solver=solver).fit(tr.X, tr.y, world=world)
    rg, rc = g.result, c.result
    assert rg.backend == "hip" and rg.transport == "loopback" and rg.converged
    tol = 1e-5 * max(1.0, abs(rc.b)) if solver == "smo" else 10 * SVMParams().tau
    assert abs(rg.b - rc.b) < tol
    assert len(set(rg.ids.tolist()) ^ set(rc.ids.tolist())) <= 2
    assert abs(g.score(te.X, te.y) - c.score(te.X, te.y)) <= 0.002
    assert {s["rank"] for s in rg.solves} == set(range(world))
    assert all(s["solver"] == solver for s in rg.solves + rc.solves)


def test_hip_cascade_one_rank_finds_the_single_gpu_svs(data):
    tr, _ = data
    g = CascadeSVM(SVMParams()).fit(tr.compact().X, tr.y, world=1, device="cuda", transport="loopback")
    s = SVC(device="cuda:0").fit(tr.compact().X, tr.y)
    assert sorted(g.result.ids.tolist()) == sorted(s.support_.tolist())
    first = g.result.solves[0]
    assert first["layer"] == "local" and first["iterations"] == s.n_iter_  # same trajectory as the SVC fit


@pytest.mark.parametrize("topology,world", [("star", 1), ("star", 3), ("tree", 2)])
def test_optimal_warm_start_skip_changes_nothing(data, monkeypatch, topology, world):
    """A solve whose warm start already meets the stop test is skipped (no Gram); the model is the
    same bit for bit as with every solve run."""
    tr, _ = data
    X = tr.compact().X
    fit = lambda: CascadeSVM(SVMParams(), topology=topology).fit(X, tr.y, world=world, device="cuda",
                                                                 transport="loopback").result
    a = fit()
    monkeypatch.setenv("SVM355_CASCADE_SKIP", "0")
    b = fit()
    assert a.ids.tolist() == b.ids.tolist() and a.b == b.b and a.rounds == b.rounds
    np.testing.assert_array_equal(a.alpha, b.alpha)
    assert not any(s["skipped"] for s in b.solves)
    skipped = [s for s in a.solves if s["skipped"]]
    if topology == "star" and world == 1:  # round 1's local solve restarts from the optimum
        assert skipped and all(s["layer"] == "local" and s["iterations"] == 1 for s in skipped)
    # every skipped solve really would have stopped at its first selection
    ref = {(s["rank"], s["round"], s["layer"]): s["iterations"] for s in b.solves}
    assert all(ref[(s["rank"], s["round"], s["layer"])] == 1 for s in skipped)


def test_serial_solve_rehearsal_with_released_grams_changes_nothing(data, monkeypatch):
    """The large-n rehearsal mode (SVM355_CASCADE_SERIAL_SOLVES=1 + SVM355_CASCADE_RELEASE_GRAM=1: each
    solve's Gram sized before its timed region and released after it, svmd_reserve_gram) times every
    solve alone and produces the same model bit for bit."""
    tr, _ = data
    X = tr.compact().X
    a = CascadeSVM(SVMParams()).fit(X, tr.y, world=3, device="cuda", transport="loopback").result
    monkeypatch.setenv("SVM355_CASCADE_SERIAL_SOLVES", "1")
    monkeypatch.setenv("SVM355_CASCADE_RELEASE_GRAM", "1")
    g = DeviceGroup(3, "loopback")  # backends read the knobs when they are created
    try:
        b = CascadeSVM(SVMParams()).fit(X, tr.y, world=3, device="cuda", group=g).result
    finally:
        g.close()
    assert a.ids.tolist() == b.ids.tolist() and a.b == b.b and a.rounds == b.rounds
    np.testing.assert_array_equal(a.alpha, b.alpha)
    assert all(s["solo_ms"] >= 0 for s in b.solves if not s["skipped"])
    assert not any(s["row_cache"] for s in b.solves)


@pytest.mark.parametrize("topology,world", [("star", 2), ("tree", 2)])
def test_row_cache_solves_equal_gram_solves(data, monkeypatch, topology, world):
    """A partition whose Gram does not fit is solved on the HBM row cache (cascade_dev.hip
    HipBackend::solve); SVM355_CASCADE_GRAM=rows forces that path.  The row-cache solver follows
    the resident-Gram trajectory bit for bit (warm starts included), so the cascade is unchanged."""
    tr, _ = data
    X = tr.compact().X
    fit = lambda: CascadeSVM(SVMParams(), topology=topology, solver="smo").fit(X, tr.y, world=world, device="cuda",
                                                                               transport="loopback").result
    a = fit()
    monkeypatch.setenv("SVM355_CASCADE_GRAM", "rows")
    b = fit()
    assert not any(s["row_cache"] for s in a.solves)
    assert all(s["row_cache"] for s in b.solves if not s["skipped"])
    assert a.ids.tolist() == b.ids.tolist() and a.b == b.b and a.rounds == b.rounds
    np.testing.assert_array_equal(a.alpha, b.alpha)
    assert [s["iterations"] for s in a.solves] == [s["iterations"] for s in b.solves]


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_rccl_group_equals_loopback(data, topology):
    tr, _ = data
    X = tr.compact().X
    a = CascadeSVM(SVMParams(), topology=topology).fit(X, tr.y, world=1, device="cuda", transport="rccl").result
    b = CascadeSVM(SVMParams(), topology=topology).fit(X, tr.y, world=1, device="cuda", transport="loopback").result
    assert a.transport == "rccl" and b.transport == "loopback"
    assert a.ids.tolist() == b.ids.tolist() and a.b == b.b and a.rounds == b.rounds
    np.testing.assert_array_equal(a.alpha, b.alpha)


def test_rccl_rank_bootstrap_equals_group(data):
    """The per-process path (ncclUniqueId -> ncclCommInitRank) with a world of one."""
    tr, _ = data
    X = tr.compact().X
    rank = RcclRank(0, RcclRank.unique_id(), 1, 0, comm_timeout_s=60)
    try:
        rank.barrier()
        a = CascadeSVM(SVMParams()).fit_rank(rank, X, tr.y, np.arange(N), N).result
    finally:
        rank.close()
    b = CascadeSVM(SVMParams()).fit(X, tr.y, world=1, device="cuda", transport="rccl").result
    assert a.ids.tolist() == b.ids.tolist() and a.b == b.b and a.rounds == b.rounds


def test_torchrun_bench_per_process_rccl_rank(data):
    """bench.py launched by torchrun (the driver's N-GPU launch), here with one process: gloo bootstrap,
    ncclUniqueId over the store, ncclCommInitRank, fit_rank, the solve-log gather and the timing max
    over ranks -- the whole per-process branch on the GPU.  Same model as the thread-rank group."""
    import os
    import socket
    import sys

    root = Path(__file__).resolve().parents[1]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=str(root))
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), str(root / "bench.py"), "--gpus", "1", "--cascade", "--rows", str(N),
           "--test-rows", str(M), "--seed", "21", "--steps", "2", "--warmup", "1", "--baseline-1gpu", "1"]
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=180)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["launch"].startswith("torchrun") and out["transport"] == "rccl" and out["n_gpus"] == 1
    tr, _ = data
    ref = CascadeSVM(SVMParams()).fit(tr.compact().X, tr.y, world=1, device="cuda", transport="rccl").result
    assert out["n_sv"] == len(ref.ids) and out["b"] == ref.b and out["rounds"] == ref.rounds
    assert out["single_gpu_s"] > 0 and out["speedup_vs_1gpu"] > 0


def test_group_keeps_working_after_a_loopback_failure(data):
    tr, _ = data
    X = tr.compact().X
    g = DeviceGroup(2, "loopback")
    try:
        with pytest.raises(NativeError, match="rank 1: injected failure"):
            CascadeSVM(SVMParams(), fail_rank=1, fail_round=1).fit(X, tr.y, world=2, device="cuda", group=g)
        r = CascadeSVM(SVMParams()).fit(X, tr.y, world=2, device="cuda", group=g).result
        assert r.converged
    finally:
        g.close()


def test_rccl_failure_aborts_the_communicator(data):
    tr, _ = data
    X = tr.compact().X
    g = DeviceGroup(1, "rccl")
    try:
        with pytest.raises(NativeError, match="rank 0: injected failure"):
            CascadeSVM(SVMParams(), fail_rank=0, fail_round=0).fit(X, tr.y, world=1, device="cuda", group=g)
        with pytest.raises(NativeError, match="aborted"):
            CascadeSVM(SVMParams()).fit(X, tr.y, world=1, device="cuda", group=g)
    finally:
        g.close()


def test_rccl_preflight_and_runtime_identity():
    """Group creation runs the preflight (every driver op with checked payloads); running it again
    explicitly passes; the RCCL runtime is identified (version + path of the loaded librccl)."""
    info = rccl_info()
    assert info["rccl_runtime"].startswith("2.") and info["rccl_path"].endswith((".so", ".so.1")) or "librccl" in \
        info["rccl_path"], info
    g = DeviceGroup(1, "rccl")
    try:
        g.exercise(preflight_script(1, 1 << 20))
        assert not g.broken
    finally:
        g.close()
    rank = RcclRank(0, RcclRank.unique_id(), 1, 0, comm_timeout_s=60)  # ncclCommInitRank + preflight
    try:
        rank.exercise(preflight_script(1, 1 << 20))
    finally:
        rank.close()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_preflight_on_device_loopback_ranks(world):
    """The preflight op set over P HIP-backend ranks sharing this GPU (strict loopback): device
    buffers, host staging, every payload checked; a mismatched sequence fails naming the ranks."""
    g = DeviceGroup(world, "loopback")
    try:
        g.exercise(preflight_script(world, 1 << 20), timeout_s=30)
        with pytest.raises(NativeError, match="mismatch"):
            g.exercise("|".join(["bc:64@0"] + ["bc:128@0"] * (world - 1)), timeout_s=10)
        g.exercise(preflight_script(world, 4096))  # loopback groups stay usable after a failure
    finally:
        g.close()


def test_shared_group_is_rebuilt_after_an_rccl_failure(data):
    """a failed RCCL fit aborts the shared group's communicators; the next fit through
    DeviceGroup.shared must build a new group instead of failing with 'create a new group'."""
    tr, _ = data
    X = tr.compact().X
    DeviceGroup.release_shared()
    with pytest.raises(NativeError, match="rank 0: injected failure"):
        CascadeSVM(SVMParams(), fail_rank=0, fail_round=0).fit(X, tr.y, world=1, device="cuda", transport="rccl")
    r = CascadeSVM(SVMParams()).fit(X, tr.y, world=1, device="cuda", transport="rccl").result
    assert r.converged and r.transport == "rccl"
    DeviceGroup.release_shared()


def _cli(tmp_path, name, *extra):
    out = tmp_path / name
    r = subprocess.run([str(EXE), "--synthetic", f"{N},{M}", "--seed", "21", "--json", str(out), "--quiet", *extra],
                       capture_output=True, text=True, timeout=240)
    return r, (json.loads(out.read_text()) if out.exists() else None)


@pytest.mark.parametrize("topology,world", [("star", 2), ("tree", 2)])
def test_native_cli_matches_python_binding(tmp_path, topology, world):
    r, nat = _cli(tmp_path, "n.json", "--topology", topology, "--gpus", str(world), "--transport", "loopback")
    assert r.returncode == 0, r.stdout + r.stderr
    tr = synthetic_mnist(N, seed=21)
    py = CascadeSVM(SVMParams(), topology=topology).fit(tr.X, tr.y, world=world, device="cuda",
                                                        transport="loopback").result
    assert nat["sv_ids"] == sorted(py.ids.tolist()) and nat["b"] == py.b and nat["rounds"] == py.rounds
    head = "modified CascadeSVM" if topology == "star" else "CascadeSVM"
    assert f"[rank 0] Running {head} with {world} processes" in r.stdout
    assert f"[rank 0] total samples = {N}, features = 784" in r.stdout
    assert "[rank 0] Final b = " in r.stdout and f"[rank 0] Cascade finished in {nat['rounds']} rounds" in r.stdout


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_native_cli_checkpoint_resume(tmp_path, topology):
    base = ["--topology", topology, "--gpus", "2", "--transport", "loopback"]
    r, full = _cli(tmp_path, "full.json", *base)
    assert r.returncode == 0, r.stderr
    ck = str(tmp_path / f"ck_{topology}")
    r, part = _cli(tmp_path, "part.json", *base, "--max-rounds", "1", "--checkpoint-dir", ck)
    assert r.returncode == 0 and part["rounds"] == 1 and not part["converged"]
    r, res = _cli(tmp_path, "res.json", *base, "--checkpoint-dir", ck, "--resume")
    assert r.returncode == 0 and "[rank 0] resumed from checkpoint at round 1" in r.stdout
    assert res["converged"] and res["rounds"] == full["rounds"]
    assert res["sv_ids"] == full["sv_ids"] and res["b"] == full["b"]


def test_native_cli_failed_rank_exits_nonzero(tmp_path):
    r, js = _cli(tmp_path, "f.json", "--gpus", "3", "--transport", "loopback", "--fail-rank", "2", "--fail-round", "1",
                 "--comm-timeout", "60")
    assert r.returncode == 1 and js is None
    assert "rank 2: injected failure at round 1" in r.stderr
