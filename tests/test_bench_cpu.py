"""bench.py's host-side logic on the CPU: the cascade critical path (the per-round slowest local
solve plus rank 0's merge; the solo device times of a serial-solve rehearsal when present), the
launch checks of ``--gpus N``, and the solve-log fields the critical path reads from the native
driver."""
import json
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from svm355 import SVMParams  # noqa: E402
from svm355.parallel.cascade import CascadeSVM, critical_path  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402


def _s(rank, rnd, layer, ms, it, solo=-1.0):
    return {"rank": rank, "round": rnd, "layer": layer, "ms": ms, "iterations": it, "solo_ms": solo}


def test_star_critical_path_takes_slowest_local_plus_merge():
    solves = [_s(0, 1, "local", 5.0, 100), _s(1, 1, "local", 7.0, 90), _s(0, 1, "merge", 3.0, 40),
              _s(0, 2, "local", 1.0, 10), _s(1, 2, "local", 2.0, 20), _s(0, 2, "merge", 0.5, 5)]
    rows, tot = critical_path(solves, "star")
    assert rows == [[1, 7.0, 3.0, 100, 40], [2, 2.0, 0.5, 20, 5]]
    assert tot == pytest.approx(12.5)


def test_tree_critical_path_takes_slowest_rank_of_every_layer():
    solves = [_s(0, 1, "layer1", 4.0, 50), _s(1, 1, "layer1", 6.0, 70), _s(2, 1, "layer1", 5.0, 60),
              _s(3, 1, "layer1", 1.0, 10), _s(0, 1, "layer2", 2.0, 30), _s(2, 1, "layer2", 3.0, 35),
              _s(0, 1, "layer4", 1.5, 20)]
    rows, tot = critical_path(solves, "tree")
    assert rows == [[1, 6.0, 4.5, 70, 55]]
    assert tot == pytest.approx(10.5)


def test_critical_path_prefers_solo_device_times():
    """A serial-solve rehearsal (SVM355_CASCADE_SERIAL_SOLVES=1) logs each solve's time alone on the
    device; the wall time of ranks sharing one GPU would overstate the P-GPU critical path."""
    solves = [_s(0, 1, "local", 50.0, 100, solo=5.0), _s(1, 1, "local", 70.0, 90, solo=7.5),
              _s(0, 1, "merge", 30.0, 40, solo=3.0)]
    rows, tot = critical_path(solves, "star")
    assert rows == [[1, 7.5, 3.0, 100, 40]]
    assert tot == pytest.approx(10.5)


def test_more_gpus_than_visible_is_refused(capsys):
    """Launched directly on a host without N GPUs, bench exits non-zero with a message (unless a
    loopback rehearsal is asked for) instead of hanging or silently running fewer ranks."""
    assert bench.main(["--gpus", "2", "--steps", "1", "--warmup", "0"]) == 2
    assert "visible GPUs" in capsys.readouterr().err


def test_cpu_solve_log_has_the_fields_the_critical_path_reads():
    tr = synthetic_mnist(600, seed=5)
    r = CascadeSVM(SVMParams(n_threads=2)).fit(tr.X, tr.y, world=2).result
    assert r.solves
    for s in r.solves:
        assert {"rank", "round", "layer", "ms", "iterations", "skipped", "row_cache", "solo_ms"} <= set(s)
        assert s["row_cache"] is False and s["solo_ms"] < 0  # CPU backend: no row cache, no solo timing
    rows, tot = critical_path(r.solves, "star")
    assert len(rows) == r.rounds and tot > 0


@pytest.mark.parametrize("topology,gpus", [("star", 2), ("tree", 4)])
def test_bench_in_process_thread_ranks_json(capsys, topology, gpus):
    """bench.main with N > 1 launched directly (no torchrun): N thread-ranks in this process (here on the
    CPU oracle: the cascade, since the distributed SMO needs GPUs).  The JSON line carries the fields
    the SCALE driver reads, and its timed region fits inside the call's wall time."""
    import json
    import time

    t0 = time.time()
    rc = bench.main(["--gpus", str(gpus), "--device", "cpu", "--rows", "1200", "--test-rows", "200", "--steps", "2",
                     "--warmup", "1", "--topology", topology, "--baseline-1gpu", "1"])
    wall = time.time() - t0
    assert rc == 0
    line = json.loads([x for x in capsys.readouterr().out.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == gpus and line["steps"] == 2 and line["warmup"] == 1
    assert line["config"]["parallelism"] == f"cascade-{topology}-dp{gpus}"
    assert line["scaling"] == "strong" and line["higher_is_better"] is False
    assert line["launch"] == "in-process thread ranks"
    assert 0 < line["ms_per_step"] * line["steps"] / 1e3 <= wall
    assert line["value"] == pytest.approx(line["ms_per_step"] / 1e3, rel=1e-3)
    assert line["speedup_vs_1gpu"] > 0 and line["single_gpu_s"] > 0
    assert line["sv_history"] and len(line["per_round_critical_path"]) == line["rounds"]
    assert line["fallback_reason"] == "cpu device"  # --parallel auto: no distributed SMO on the CPU
    assert line["transport"] == "loopback"


def test_bench_smo_refuses_cpu(capsys):
    assert bench.main(["--gpus", "2", "--device", "cpu", "--parallel", "smo", "--rows", "600", "--steps", "1"]) == 2
    assert "needs uint8 pixel rows on GPUs" in capsys.readouterr().err


def test_bench_decomp_solver_needs_gpus_and_its_own_parallel_mode(capsys):
    """The decomposition solver (the GPU default, every cascade solve too) runs on GPUs; the CPU oracle
    and the distributed pairwise SMO (--parallel smo) belong to --solver smo."""
    assert bench.main(["--solver", "decomp", "--device", "cpu", "--rows", "600", "--steps", "1"]) == 2
    assert "runs on GPUs" in capsys.readouterr().err
    assert bench.main(["--solver", "decomp", "--gpus", "2", "--parallel", "smo", "--transport", "loopback",
                       "--rows", "600"]) == 2


def test_bench_parallel_decomp_cpu_twin_thread_ranks(capsys):
    """--device cpu --parallel decomp: the distributed decomposition's CPU twin on thread ranks (strict
    loopback), bit-identical to the one-rank oracle solve."""
    assert bench.main(["--gpus", "2", "--device", "cpu", "--parallel", "decomp", "--rows", "600", "--steps", "1",
                       "--baseline-1gpu", "1"]) == 0
    out = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1])
    assert out["config"]["parallelism"] == "distributed-decomp-dp2"
    assert out["launch_form"] == "thread ranks on the CPU oracle (loopback)"
    assert out["bit_identical_to_1gpu"] is True and out["stop_reason"] == "converged"


def test_bench_hostcomm_needs_torchrun(capsys):
    assert bench.main(["--gpus", "2", "--transport", "hostcomm", "--parallel", "decomp", "--rows", "600"]) == 2
    assert "--transport hostcomm is a per-process transport" in capsys.readouterr().err


def test_bench_max_iter_and_rows_away_from_60k(capsys):
    """--max-iter reaches the timed solve (here the CPU oracle ends on the cap), and a row count other
    than the reference's 60k names itself in the config with no reference-relative figures."""
    assert bench.main(["--device", "cpu", "--rows", "900", "--test-rows", "100", "--steps", "1", "--warmup", "0",
                       "--max-iter", "20"]) == 0
    out = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1])
    assert out["stop_reason"] == "max_iter" and out["iterations"] <= 21
    assert "900 rows" in out["config"]["model"] and out["config"]["global_batch"] == 900
    assert out["vs_baseline"] is None and out["speedup_vs_serial"] is None
