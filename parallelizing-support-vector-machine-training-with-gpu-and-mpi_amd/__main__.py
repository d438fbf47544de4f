"""Command-line entry points: ``python -m svm355 {serial,gpu,sweep,cascade,scale,multiclass} [options]``.

serial   the reference's serial program (code/main3.cpp) -> native ``bin/svm_serial``
gpu      the single-GPU program (code/gpu_svm_main3.cu; ``--n-limit N`` = gpu_svm_main4.cu) ->
         native ``bin/svm_gpu``
sweep    the training-set-size sweep of code/gpu_svm4.sh (n = 10k, 20k, ..., 60k on one GPU),
         printing the reference's Table 2 layout (training / prediction seconds per n)
cascade  the MPI Cascade programs (code/mpi_svm_main2.cpp ``--topology star`` = modified two-layer,
         code/mpi_svm_main3.cpp ``--topology tree`` = classical) on the native driver: ``--gpus P``
         thread-ranks, one GPU and one RCCL communicator each (ncclCommInitAll, xGMI), or ``--cpu``
         thread-ranks on the C++ oracle.  stdout follows the reference's ``[rank 0] ...`` lines
         (SURVEY §5.5).  ``--native`` runs the C++ CLI bin/svm_cascade (same driver, no Python).

scale    the rank-count sweep of code/mpi_svm2.sh / mpi_svm3.sh (``mpirun -np P`` for each P), for
         every training size of ``--sizes`` (default 60000 and 1000000): the N-GPU trainer at P = 1,
         2, 4, 8 ... ranks (one GPU each; ``--transport loopback`` rehearses P ranks on fewer GPUs
         and times every rank's device work alone, so the critical path of P GPUs is measured) --
         ``--trainer decomp`` (default): the distributed decomposition solver, bit-identical to one
         GPU; ``--trainer cascade``: the reference's Cascade SVM (``--topology star|tree``) -- next to
         the single-GPU trainer on the same data, in the reference's Table 3 / 4 layout

multiclass  all-digit one-vs-rest (models/multiclass.py): one shared Gram per GPU, class solves
         concurrent on streams; ``--gpus P`` deals the classes over P ranks (torchrun, RCCL).

The native CLIs take the options listed in ``csrc/apps/cli_common.h`` (``--dataset``,
``--synthetic N[,M]``, ``--C``, ``--gamma``, ``--tau``, ``--model-dir``, ``--json`` ...).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import subprocess
import sys
import time
from pathlib import Path

PKG = Path(__file__).resolve().parent
# A rank that dies leaves the others blocked in a collective: the process group's watchdog aborts
# the job after this long instead of hanging it.
COLLECTIVE_TIMEOUT = datetime.timedelta(minutes=10)


def _native(name: str, args) -> int:
    exe = PKG / "bin" / name
    if not exe.exists():
        from . import build

        build.build_all(hip=name != "svm_serial")
    return subprocess.call([str(exe), *args])


def _sweep(argv) -> int:
    ap = argparse.ArgumentParser(prog="svm355 sweep", description="gpu_svm4.sh: n = 10k..60k on one GPU")
    ap.add_argument("--sizes", default="10000,20000,30000,40000,50000,60000")
    ap.add_argument("--out", default=None, help="write the per-n JSON summaries to this file")
    a, rest = ap.parse_known_args(argv)
    exe = PKG / "bin" / "svm_gpu"
    if not exe.exists():
        from . import build

        build.build_all()
    rows = []
    tmp = Path(os.environ.get("TMPDIR", "/tmp")) / f"svm355_sweep_{os.getpid()}.json"
    for n in [int(v) for v in a.sizes.split(",")]:
        rc = subprocess.call([str(exe), "--n-limit", str(n), "--json", str(tmp), "--quiet", *rest],
                             stdout=subprocess.DEVNULL)
        if rc:
            return rc
        rows.append(json.loads(tmp.read_text()))
    tmp.unlink(missing_ok=True)
    print(f"{'n train':>8} {'train (s)':>10} {'predict (s)':>12} {'iterations':>11} {'#SV':>6} {'accuracy':>9} gram")
    for r in rows:
        print(f"{r['n']:>8} {r['training_ms'] / 1e3:>10.3f} {r['prediction_ms'] / 1e3:>12.3f} {r['iterations']:>11} "
              f"{r['n_sv']:>6} {r['accuracy']:>9.4f} {r.get('gram_path', '')}")
    if a.out:
        Path(a.out).write_text(json.dumps(rows, indent=1) + "\n")
    return 0


def _cascade(argv) -> int:
    ap = argparse.ArgumentParser(prog="svm355 cascade", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--topology", choices=["star", "tree"], default="star",
                    help="star = modified two-layer (mpi_svm_main2), tree = classical (mpi_svm_main3)")
    ap.add_argument("--dataset", default="mnist3", help="CSV prefix: P_train_data.csv / P_test_data.csv")
    ap.add_argument("--train", default=None)
    ap.add_argument("--test", default=None)
    ap.add_argument("--synthetic", default=None, help="N[,M]: MNIST-shaped synthetic data instead of CSVs")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--positive-label", type=int, default=1)
    ap.add_argument("--C", type=float, default=10.0)
    ap.add_argument("--gamma", type=float, default=0.00125)
    ap.add_argument("--tau", type=float, default=1e-5)
    ap.add_argument("--max-rounds", type=int, default=50)
    ap.add_argument("--wss", choices=["first", "second"], default="first",
                    help="working-set selection: first order (the reference) or the opt-in second-order choice")
    ap.add_argument("--solver", choices=["auto", "decomp", "smo"], default="auto",
                    help="every local / merge solve: the warm-started working-set decomposition (decomp), the "
                         "reference's pairwise SMO (smo), or auto: on GPUs per solve (the decomposition for cold and "
                         "small sets, the pairwise SMO for large warm-started ones), on --cpu the pairwise oracle")
    ap.add_argument("--cpu", action="store_true", help="CPU thread-ranks on the native oracle instead of GPUs")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU; thread-ranks of this process)")
    ap.add_argument("--transport", choices=["auto", "rccl", "loopback"], default="auto",
                    help="GPU ranks: RCCL (one GPU per rank) or loopback (ranks share GPUs, host-staged)")
    ap.add_argument("--model-dir", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--checkpoint-dir", default=None, help="per-round cascade state (resume with --resume)")
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--comm-timeout", type=float, default=600.0, help="deadline of one exchange (s)")
    ap.add_argument("-v", "--verbose", type=int, default=1)
    ap.add_argument("--native", action="store_true", help="run the C++ CLI bin/svm_cascade instead")
    a = ap.parse_args(argv)

    if a.native:
        args = ["--topology", a.topology, "--gpus", str(max(1, a.gpus)), "--transport", a.transport,
                "--max-rounds", str(a.max_rounds), "--C", str(a.C), "--gamma", str(a.gamma), "--tau", str(a.tau),
                "--positive-label", str(a.positive_label), "--seed", str(a.seed), "--comm-timeout", str(a.comm_timeout),
                "--wss", a.wss, "--solver", a.solver]
        if a.synthetic:
            args += ["--synthetic", a.synthetic]
        else:
            args += ["--train", a.train or f"{a.dataset}_train_data.csv", "--test", a.test or f"{a.dataset}_test_data.csv"]
        if a.json:
            args += ["--json", a.json]
        if a.model_dir:
            args += ["--model-dir", a.model_dir]
        if a.checkpoint_dir:
            args += ["--checkpoint-dir", a.checkpoint_dir] + (["--resume"] if a.resume else [])
        return _native("svm_cascade", args)

    from .parallel.cascade import CascadeSVM
    from .utils.config import SVMParams, default_threads
    from .utils.data import load_csv, synthetic_mnist

    if a.synthetic:
        parts = a.synthetic.split(",")
        n_total, m = int(parts[0]), int(parts[1]) if len(parts) > 1 else 10000
        tr = synthetic_mnist(n_total, seed=a.seed, positive_label=a.positive_label)
        te = synthetic_mnist(m, seed=a.seed, offset=n_total, positive_label=a.positive_label)
    else:
        tr = load_csv(a.train or f"{a.dataset}_train_data.csv", positive_label=a.positive_label)
        te = load_csv(a.test or f"{a.dataset}_test_data.csv", positive_label=a.positive_label)
    if tr.n == 0:
        print("Error: No data read from file.", file=sys.stderr)
        return 1
    # Launched by torchrun (``torchrun --nproc-per-node P -m svm355 cascade ...``, the reference's
    # ``mpirun -np P``): this process is one rank -- its GPU LOCAL_RANK over RCCL (ncclCommInitRank), or
    # with --cpu the C++ oracle over the launcher's gloo group -- and trains on its contiguous partition.
    per_process = "LOCAL_RANK" in os.environ and "WORLD_SIZE" in os.environ
    world = int(os.environ["WORLD_SIZE"]) if per_process else max(1, a.gpus)
    params = SVMParams(C=a.C, gamma=a.gamma, tau=a.tau, n_threads=max(1, default_threads() // world),
                       wss=2 if a.wss == "second" else 1)
    model = CascadeSVM(params, topology=a.topology, max_rounds=a.max_rounds, verbose=a.verbose,
                       checkpoint_dir=a.checkpoint_dir, resume=a.resume, comm_timeout_s=a.comm_timeout,
                       solver=a.solver)
    device = "cpu" if a.cpu else "cuda"
    X = tr.X if a.cpu else tr.compact().X
    crank = None
    if per_process:
        import numpy as np
        import torch.distributed as dist

        from .parallel.cascade import partition_bounds

        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=max(60.0, a.comm_timeout)))
        if a.cpu:
            from .parallel.hostcomm import HostCommRank

            crank = HostCommRank()
        else:
            from .parallel.rccl import RcclRank

            crank = RcclRank.from_torch_dist(int(os.environ["LOCAL_RANK"]), a.comm_timeout)
        lo, hi = partition_bounds(tr.n, world, crank.rank)
        t0 = time.perf_counter()
        model.fit_rank(crank, X[lo:hi], tr.y[lo:hi], np.arange(lo, hi), tr.n)
    else:
        t0 = time.perf_counter()
        model.fit(X, tr.y, world=world, device=device, transport=a.transport)
    t1 = time.perf_counter()
    res = model.result
    if crank is not None and crank.rank != 0:  # the reference prints and saves on rank 0 only
        crank.close()
        dist.destroy_process_group()
        return 0
    acc = None
    if te.n:
        correct = int(round(model.score(te.X, te.y) * te.n))
        acc = correct / te.n
        print(f"[rank 0] Test accuracy (final model) = {acc} ({correct}/{te.n})")
    else:
        print("[rank 0] No test data found or test file empty.")
    t2 = time.perf_counter()
    pred_ms = (t2 - t1) * 1e3
    print(f"[rank 0] Final global SV count = {len(res.ids)}")
    print(f"[rank 0] Cascade finished in {res.rounds} rounds")
    print(f"[rank 0] training time = {int(res.train_ms)} ms")
    print(f"[rank 0] prediction time = {int(pred_ms)} ms")
    print(f"[rank 0] elapsed time = {int(res.train_ms + pred_ms)} ms")
    if a.json:
        out = {"program": f"svm355 cascade ({a.topology})", "n": tr.n, **model.summary(), "accuracy": acc,
               "training_ms": res.train_ms, "prediction_ms": pred_ms, "fit_wall_ms": (t1 - t0) * 1e3,
               "solves": res.solves}
        Path(a.json).write_text(json.dumps(out) + "\n")
    if a.model_dir:
        model.save(a.model_dir)
    if crank is not None:
        crank.close()
        dist.destroy_process_group()
    return 0


# The reference cascades' training times at P ranks (MPI on CPUs) and its
# serial SMO time at 60k (Table 1).
REF_CASCADE_S = {"star": {4: 886.733, 8: 649.773, 16: 440.705, 32: 333.696, 64: 301.263},
                 "tree": {4: 1194.269, 8: 839.406, 16: 662.153, 32: 671.448, 64: 673.580}}
REF_SERIAL_60K_S = 3285.662


def _scale(argv) -> int:
    ap = argparse.ArgumentParser(prog="svm355 scale", description="mpi_svm2.sh / mpi_svm3.sh over rank counts")
    ap.add_argument("--ranks", default="1,2,4,8", help="comma-separated rank counts P")
    ap.add_argument("--trainer", choices=["decomp", "cascade"], default="decomp",
                    help="the distributed decomposition solver (default; the one-GPU trainer's trajectory on P "
                         "GPUs) or the reference's Cascade SVM")
    ap.add_argument("--topology", choices=["star", "tree"], default="star")
    ap.add_argument("--sizes", default="60000,1000000", help="comma-separated training sizes N (synthetic)")
    ap.add_argument("--synthetic", default=None, help="N[,M]: one MNIST-shaped synthetic size (overrides --sizes)")
    ap.add_argument("--test-rows", type=int, default=10000)
    ap.add_argument("--train", default=None, help="reference CSV (instead of synthetic data)")
    ap.add_argument("--test", default=None)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--cpu", action="store_true", help="CPU thread-ranks on the native oracle")
    ap.add_argument("--transport", choices=["auto", "rccl", "loopback"], default="auto",
                    help="rccl: one GPU per rank (P > visible GPUs is skipped); loopback: P ranks share the "
                         "visible GPUs and every rank's device work is also timed alone (critical path)")
    ap.add_argument("--repeats", type=int, default=3, help="timed fits per P (median reported)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--comm-timeout", type=float, default=120.0)
    ap.add_argument("--max-iter", type=int, default=100000,
                    help="pair-update cap of every solve (the reference's 100,000; large n needs more)")
    ap.add_argument("--json", default=None, help="write the per-size, per-P rows to this file")
    a = ap.parse_args(argv)
    ranks = [int(v) for v in a.ranks.split(",")]
    if a.transport == "loopback" and not a.cpu:
        os.environ["SVM355_CASCADE_SERIAL_SOLVES"] = "1"  # read when the rank backends are created
    if a.cpu and a.trainer == "decomp":
        print("svm355 scale: the CPU oracle of the decomposition holds an n x n kernel matrix; use "
              "--trainer cascade with --cpu", file=sys.stderr)
        return 2

    import numpy as np

    from .models.svc import SVC
    from .parallel.cascade import CascadeSVM, critical_path
    from .parallel.decomp import DistributedDecompSVC
    from .utils.config import SVMParams, default_threads
    from .utils.data import load_csv, synthetic_mnist

    ndev = 0
    if not a.cpu:
        import torch

        ndev = torch.cuda.device_count()
        if ndev < 1:
            print("svm355 scale: no GPU visible (use --cpu)", file=sys.stderr)
            return 2

    def timed(fn):
        for _ in range(a.warmup):
            fn()
        ts = []
        for _ in range(max(1, a.repeats)):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    if a.train:
        datasets = [(load_csv(a.train), load_csv(a.test) if a.test else None)]
    else:
        if a.synthetic:
            parts = a.synthetic.split(",")
            sizes, m = [int(parts[0])], int(parts[1]) if len(parts) > 1 else a.test_rows
        else:
            sizes, m = [int(v) for v in a.sizes.split(",")], a.test_rows
        datasets = [(synthetic_mnist(n, seed=a.seed), synthetic_mnist(m, seed=a.seed, offset=n)) for n in sizes]
    from .parallel.rccl import DeviceGroup

    out_sizes = []
    for tr, te in datasets:
        X = tr.X if a.cpu else tr.compact().X  # pixels travel as uint8, widened on the device
        # the single-device baseline: the GPU trainer (cuda:0) or the serial oracle
        base_dev = "cpu" if a.cpu else "cuda:0"
        single = SVC(device=base_dev, max_iter=a.max_iter)
        t_single = timed(lambda: single.fit(X, tr.y))
        rows = []
        for P in ranks:
            if not a.cpu and a.transport in ("auto", "rccl") and P > ndev:
                print(f"svm355 scale: P = {P} needs {P} GPUs ({ndev} visible), skipped "
                      "(--transport loopback rehearses it on the visible GPUs)", file=sys.stderr)
                continue
            if a.trainer == "cascade" and a.topology == "tree" and P & (P - 1):
                print(f"svm355 scale: the tree cascade needs a power-of-2 P, {P} skipped", file=sys.stderr)
                continue
            group = None if a.cpu else DeviceGroup(P, a.transport, a.comm_timeout)
            try:
                if a.trainer == "decomp":
                    model = DistributedDecompSVC(P, group=group, max_iter=a.max_iter)
                    t = timed(lambda: model.fit(X, tr.y))
                    solo = model.solo_
                    row = {"P": P, "train_s": round(t, 6), "outer_iterations": model.stats_["outer_iterations"],
                           "iterations": int(model.n_iter_), "n_sv": int(len(model.support_)), "b": model.b_,
                           "bit_identical_to_1gpu": bool(model.n_iter_ == single.n_iter_ and model.b_ == single.b_
                                                         and np.array_equal(model.alpha_, single.alpha_)),
                           "critical_path_solve_ms": solo["critical_path_ms"] if solo else None,
                           "critical_path_basis": "solo device time per rank segment" if solo else None,
                           "solo": solo, "accuracy": model.score(te.X, te.y) if te is not None and te.n else None,
                           "transport": group.transport if group is not None else "cpu"}
                else:
                    threads = max(1, default_threads() // P) if a.cpu else default_threads()
                    model = CascadeSVM(SVMParams(n_threads=threads, max_iter=a.max_iter), topology=a.topology,
                                       comm_timeout_s=a.comm_timeout)
                    t = timed(lambda: model.fit(X, tr.y, world=P, device="cpu" if a.cpu else "cuda", group=group))
                    r = model.result
                    _, crit_ms = critical_path(r.solves, a.topology)
                    row = {"P": P, "train_s": round(t, 6), "driver_train_ms": round(r.train_ms, 3),
                           "critical_path_solve_ms": crit_ms,
                           "critical_path_basis": "solo device time per solve"
                           if any(s.get("solo_ms", -1.0) >= 0 for s in r.solves) else "wall time per solve",
                           "rounds": r.rounds, "converged": r.converged, "n_sv": int(len(r.ids)), "b": r.b,
                           "rank0_smo_iterations": int(sum(s["iterations"] for s in r.solves if s["rank"] == 0)),
                           "accuracy": model.score(te.X, te.y) if te is not None and te.n else None,
                           "transport": r.transport}
                    ref = REF_CASCADE_S[a.topology].get(P)
                    if ref and tr.n == 60000:
                        row["speedup_vs_ref_cascade_same_P"] = round(ref / t, 2)
            finally:
                if group is not None:
                    group.close()
            eff_t = row["critical_path_solve_ms"] / 1e3 if (a.transport == "loopback" and row["critical_path_solve_ms"]) \
                else t
            row.update(speedup_vs_single=round(t_single / eff_t, 4), efficiency_vs_single=round(t_single / eff_t / P, 4))
            if tr.n == 60000:
                row["speedup_vs_ref_serial"] = round(REF_SERIAL_60K_S / eff_t, 2)
            rows.append(row)
        acc1 = single.score(te.X, te.y) if te is not None and te.n else None
        what = "distributed decomposition" if a.trainer == "decomp" else f"{a.topology} cascade"
        print(f"n = {tr.n}: single {'CPU oracle' if a.cpu else 'GPU trainer'}: {t_single:.4f} s, {single.n_iter_} "
              f"iterations, {len(single.support_)} SVs, accuracy {acc1}; {what} per P "
              f"({'speed-ups from the solo-timed critical path' if a.transport == 'loopback' else 'wall time'}):")
        print(f"{'P':>3} {'train (s)':>10} {'crit. path (s)':>15} {'vs single':>10} {'efficiency':>11} {'#SV':>6} "
              f"{'accuracy':>9}")
        for r in rows:
            acc = f"{r['accuracy']:.4f}" if r["accuracy"] is not None else "-"
            cp = f"{r['critical_path_solve_ms'] / 1e3:.4f}" if r["critical_path_solve_ms"] else "-"
            print(f"{r['P']:>3} {r['train_s']:>10.4f} {cp:>15} {r['speedup_vs_single']:>10.3f} "
                  f"{r['efficiency_vs_single']:>11.3f} {r['n_sv']:>6} {acc:>9}")
        out_sizes.append({"n": tr.n, "single_s": t_single, "single_iterations": int(single.n_iter_),
                          "single_n_sv": int(len(single.support_)), "single_accuracy": acc1, "rows": rows})
    if a.json:
        Path(a.json).write_text(json.dumps({
            "program": f"svm355 scale ({a.trainer if a.trainer == 'decomp' else a.topology + ' cascade'})",
            "device": "cpu" if a.cpu else "cuda:0", "transport": a.transport, "sizes": out_sizes}) + "\n")
    return 0


def _launch_self(cmd: str, argv, gpus: int) -> int:
    """Start torchrun with ``gpus`` ranks running ``python -m svm355 <cmd>`` (a child process)."""
    fwd, skip = [], False
    for x in argv:
        if skip:
            skip = False
        elif x == "--gpus":
            skip = True
        elif not x.startswith("--gpus="):
            fwd.append(x)
    run = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29533"),
           "-m", "svm355", cmd, *fwd]
    return subprocess.call(run, cwd=str(PKG.parent))


def _multiclass(argv) -> int:
    ap = argparse.ArgumentParser(prog="svm355 multiclass")
    ap.add_argument("--dataset", default="mnist3")
    ap.add_argument("--train", default=None)
    ap.add_argument("--test", default=None)
    ap.add_argument("--synthetic", default=None, help="N[,M]: MNIST-shaped synthetic data")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--C", type=float, default=10.0)
    ap.add_argument("--gamma", type=float, default=0.00125)
    ap.add_argument("--tau", type=float, default=1e-5)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--solver", choices=["auto", "batched", "streams", "decomp"], default="auto",
                    help="GPU class solves: one batched pairwise launch over a shared Gram (auto), or the "
                         "decomposition solver per class with no Gram (decomp)")
    ap.add_argument("--gpus", type=int, default=0, help="launch torchrun with this many ranks (classes dealt over them)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl")
    ap.add_argument("--model-dir", default=None, help="save the model (one directory of reference model files per class)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    if "RANK" not in os.environ and a.gpus > 1:
        return _launch_self("multiclass", argv, a.gpus)

    import numpy as np
    import torch
    import torch.distributed as dist

    from .models.multiclass import OneVsRestSVC
    from .parallel.transport import TorchDistTransport
    from .utils.data import load_csv, synthetic_mnist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    use_gpu = not a.cpu and torch.cuda.is_available()
    dev = "cpu"
    if use_gpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
        dev = f"cuda:{torch.cuda.current_device()}"
    transport = None
    if world > 1:
        backend = a.backend if use_gpu else "gloo"
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(dev), timeout=COLLECTIVE_TIMEOUT)
        else:
            dist.init_process_group("gloo", timeout=COLLECTIVE_TIMEOUT)
        transport = TorchDistTransport(torch.device(dev) if backend == "nccl" else torch.device("cpu"))
    if a.synthetic:
        parts = a.synthetic.split(",")
        n, m = int(parts[0]), int(parts[1]) if len(parts) > 1 else 10000
        tr, te = synthetic_mnist(n, seed=a.seed), synthetic_mnist(m, seed=a.seed, offset=n)
    else:
        tr = load_csv(a.train or f"{a.dataset}_train_data.csv")
        te = load_csv(a.test or f"{a.dataset}_test_data.csv")
    model = OneVsRestSVC(C=a.C, gamma=a.gamma, tol=a.tau, device=dev, solver=a.solver if use_gpu else "auto")
    t0 = time.perf_counter()
    model.fit(tr.X, tr.labels, transport=transport)
    if use_gpu:
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    acc = model.score(te.X, te.labels) if te.n else None
    t2 = time.perf_counter()
    if rank == 0:
        print(f"[rank 0] one-vs-rest over {len(model.classes_)} classes on {world} rank(s), n = {tr.n}")
        print(f"[rank 0] union SV count = {len(model.support_)}, iterations per class = {model.n_iter_.tolist()}")
        print(f"[rank 0] Test accuracy = {acc}")
        print(f"[rank 0] training time = {int((t1 - t0) * 1e3)} ms, prediction time = {int((t2 - t1) * 1e3)} ms")
        if a.model_dir:
            model.save(a.model_dir)
        if a.json:
            Path(a.json).write_text(json.dumps({
                "program": "svm355 multiclass", "world": world, "n": tr.n, "classes": model.classes_.tolist(),
                "n_sv_union": int(len(model.support_)), "n_iter": model.n_iter_.tolist(),
                "b": model.intercepts_b_.tolist(), "stop_reasons": model.stop_reasons_, "accuracy": acc,
                "solver": getattr(model, "timings_", {}).get("smo_solver", "cpu"),
                "training_ms": (t1 - t0) * 1e3, "prediction_ms": (t2 - t1) * 1e3}) + "\n")
    if world > 1:
        dist.destroy_process_group()
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    cmd, rest = argv[0], argv[1:]
    if cmd == "serial":
        return _native("svm_serial", rest)
    if cmd == "gpu":
        return _native("svm_gpu", rest)
    fn = {"sweep": _sweep, "cascade": _cascade, "multiclass": _multiclass, "scale": _scale}.get(cmd)
    if fn is None:
        print(f"unknown command {cmd!r}\n\n{__doc__}", file=sys.stderr)
        return 2
    try:
        return fn(rest)
    except ValueError as e:  # a bad input or configuration (the reference MPI_Aborts with a message): no traceback
        print(f"svm355 {cmd}: {e}", file=sys.stderr)
        return 2


if __name__ == "__main__":
    sys.exit(main())
