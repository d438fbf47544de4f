#!/usr/bin/env python3
"""Headline benchmark: SMO train time on the MNIST-60k one-vs-rest RBF config (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 60000] [--topology star|tree]

One "step" is one complete training run on the fixed synthetic 60k x 784 MNIST-shaped matrix
(an SVM has no random init; the data are a deterministic synthetic draw of MNIST's shape and value
domain because MNIST itself is not available offline):

* N = 1: the single-GPU trainer (gpu_svm_main3.cu equivalent).  Timed scope = the reference's GPU
  "training" scope (gpu_svm_main3.cu:525-616): H2D of X and y, min/max + scaling, RBF Gram, device
  SMO to convergence.  Rows are held as uint8 (what MNIST is) and widened to FP64 on the device,
  where every value is exact (``--input f64`` ships FP64 rows like the reference, same results).
* N > 1: the Cascade SVM (modified two-layer star, mpi_svm_main2.cpp, default; ``--topology tree`` =
  classical mpi_svm_main3.cpp) on N GPUs, one rank per GPU, RCCL over xGMI, all on the ONE native
  driver (csrc/cascade):
    - launched directly (``python bench.py --gpus N``): N thread-ranks of this process, one GPU and
      one communicator each (ncclCommInitAll) — nothing is re-launched;
    - launched by torchrun (WORLD_SIZE = N): one rank per process on GPU LOCAL_RANK; the
      ncclUniqueId travels over the launcher's store (gloo group), ncclCommInitRank.
  Timed scope = a whole cascade fit: each rank's H2D of its partition, global scaling, all rounds to
  convergence, the final model on the host.

The timed region is bracketed by a barrier + device synchronisation on both sides and the maximum
over ranks is reported.  value = seconds per training run (lower is better); vs_baseline = value /
58.570 s (the reference's single-GPU SMO time).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

import numpy as np

# RCCL between processes (torchrun ranks) needs dmabuf IPC; the legacy IPC mode fails with
# "hipIpcGetMemHandle: invalid argument" on these hosts.  Must be set before the HSA runtime starts.
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

REF_GPU_S = 58.570  # GPU SMO training time, 60k
REF_SERIAL_S = 3285.662  # serial SMO training time, 60k
REF_GPU_PRED_S = 38.297  # GPU prediction time, 60k train / 10k test
REF_STAR_S = {4: 886.733, 8: 649.773, 16: 440.705, 32: 333.696, 64: 301.263}
REF_TREE_S = {4: 1194.269, 8: 839.406, 16: 662.153, 32: 671.448, 64: 673.580}
METRIC = "SMO train time (s) + speedup vs serial, MNIST-60k RBF; accuracy/#SV parity"


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    # --rows / --test-rows: spellings torchrun's own parser does not take for an abbreviation of its options
    ap.add_argument("--n", "--rows", dest="n", type=int, default=60000, help="training rows (MNIST-60k config)")
    ap.add_argument("--m", "--test-rows", dest="m", type=int, default=10000, help="test rows for the parity fields")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--topology", choices=["star", "tree"], default="star")
    ap.add_argument("--transport", choices=["auto", "rccl", "loopback"], default="auto",
                    help="direct launch, N > 1: rccl (one GPU per rank) or loopback (a rehearsal of N ranks "
                         "sharing the visible GPUs, host-staged exchanges)")
    ap.add_argument("--input", choices=["u8", "f64"], default="u8",
                    help="host row format: uint8 pixels (default) or FP64 as in the reference")
    ap.add_argument("--cascade", action="store_true", help="run the cascade even with one GPU")
    ap.add_argument("--baseline-1gpu", type=int, default=3,
                    help="N > 1: single-GPU fits timed after the cascade for speedup_vs_1gpu (0 = skip)")
    ap.add_argument("--wss", choices=["first", "second"], default="first",
                    help="working-set selection: first order (the reference; the headline) or the opt-in second-order")
    ap.add_argument("--comm-timeout", type=float, default=120.0,
                    help="N > 1: seconds any rank waits on an exchange before every rank aborts its communicator "
                         "(a fit takes well under a second; a dead peer must not hang the run)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: the same launch paths on the C++ oracle (CPU tests of the torchrun / thread-rank "
                         "plumbing; N > 1 under torchrun exchanges over gloo); not a benchmark")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    a = ap.parse_args(argv)

    import torch

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per process under torchrun; with one process (--cascade) the same per-process path runs
    # on a single GPU, so a one-GPU box rehearses the launch the N-GPU run takes
    multiproc = world_env > 1 or ("LOCAL_RANK" in os.environ and a.cascade)
    if multiproc and world_env != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        return 2
    cpu = a.device == "cpu"
    ndev = torch.cuda.device_count() if not cpu else 1 << 30  # does not initialise the GPU on this image
    if not multiproc and a.gpus > 1 and a.transport != "loopback" and ndev < a.gpus:
        print(f"bench.py: --gpus {a.gpus} needs {a.gpus} visible GPUs, {ndev} visible "
              "(use --transport loopback for a one-GPU rehearsal)", file=sys.stderr)
        return 2
    if multiproc and ndev <= local_rank:
        print(f"bench.py: LOCAL_RANK {local_rank} but {ndev} visible GPUs", file=sys.stderr)
        return 2

    from svm355 import SVC, SVMParams
    from svm355.parallel.cascade import CascadeSVM, critical_path, partition_bounds
    from svm355.utils.data import synthetic_mnist

    dev_index = local_rank if multiproc else 0
    if not cpu:
        torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index) if not cpu else torch.device("cpu")
    sync = (lambda: torch.cuda.synchronize(dev)) if not cpu else (lambda: None)
    use_cascade = a.gpus > 1 or a.cascade
    dist = None
    if multiproc:
        import torch.distributed as dist

        dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=10))  # bootstrap store + timing max

    params = SVMParams(wss=2 if a.wss == "second" else 1)
    te = synthetic_mnist(a.m, seed=a.seed, offset=a.n) if rank == 0 else None
    if multiproc:
        lo, hi = partition_bounds(a.n, world_env, rank)
        tr = synthetic_mnist(hi - lo, seed=a.seed, offset=lo)
    else:
        tr = synthetic_mnist(a.n, seed=a.seed)
    if a.input == "u8":
        tr = tr.compact()
        te = te.compact() if te is not None else None

    group = crank = None
    if use_cascade:
        if multiproc and cpu:
            from svm355.parallel.hostcomm import HostCommRank

            crank = HostCommRank()
        elif multiproc:
            from svm355.parallel.rccl import RcclRank

            crank = RcclRank.from_torch_dist(dev_index, a.comm_timeout)
        elif not cpu:
            from svm355.parallel.rccl import DeviceGroup

            group = DeviceGroup(a.gpus, a.transport, a.comm_timeout)

    def barrier_sync():
        sync()
        if crank is not None:
            crank.barrier()  # RCCL all-reduce over the cascade's own communicators
        if dist is not None:
            dist.barrier()
        sync()

    model = None

    def step():
        nonlocal model
        if not use_cascade:
            model = SVC(device=str(dev), wss=a.wss).fit(tr.X, tr.y)
        elif multiproc:
            model = CascadeSVM(params, topology=a.topology, comm_timeout_s=a.comm_timeout).fit_rank(
                crank, tr.X, tr.y, np.arange(lo, hi), a.n)
        else:
            model = CascadeSVM(params, topology=a.topology, comm_timeout_s=a.comm_timeout).fit(
                tr.X, tr.y, world=a.gpus, device="cpu" if cpu else "cuda", group=group)

    warm_ms = []
    for _ in range(a.warmup):
        tw = time.perf_counter()
        step()
        sync()
        warm_ms.append(round((time.perf_counter() - tw) * 1e3, 3))
    barrier_sync()
    t0 = time.perf_counter()
    marks, parts = [], []
    for _ in range(a.steps):
        step()
        marks.append(time.perf_counter())  # host-side step boundaries (diagnostic only)
        if not use_cascade:  # per-step upload / Gram / SMO split (diagnostic only)
            parts.append([round(model.timings_.get(k, 0.0), 2) for k in ("upload_preprocess_ms", "gram_alloc_ms",
                                                                           "gram_ms", "smo_ms")]
                         + [round(model.fit_time_ * 1e3, 2)])
    barrier_sync()
    elapsed = time.perf_counter() - t0
    step_ms = [round((b - a_) * 1e3, 3) for a_, b in zip([t0] + marks[:-1], marks)]
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    ms = elapsed / a.steps * 1e3
    value = ms / 1e3
    extra = {}
    if not use_cascade:
        # Prediction on the 10k test rows (outside the timed region): H2D, scaling with the training
        # statistics, MFMA cross-kernel against the SVs, decision values back to the host.  The
        # reference's GPU "prediction" (38.3 s at 60k) also parses the test CSV.
        sync()
        tp = time.perf_counter()
        model.decision_function(te.X)
        sync()
        pred_ms = (time.perf_counter() - tp) * 1e3
        acc = model.score(te.X, te.y)
        extra = {"n_sv": int(len(model.support_)), "iterations": int(model.n_iter_), "b": float(model.b_),
                 "accuracy": acc, "stop_reason": model.stop_reason_, "timings_ms": model.timings_,
                 "prediction_ms_10k": round(pred_ms, 3), "ref_gpu_prediction_s": REF_GPU_PRED_S,
                 "warmup_fit_ms": warm_ms,
                 "caveats": "timed fits reuse the library's grow-only Gram buffer and device context, allocated by "
                            "the first (warm-up) fit, whose time is warmup_fit_ms[0]; host rows are uint8 pixels "
                            "widened to fp64 on the device (bit-identical results to --input f64, which ships fp64 "
                            "rows like the reference); the data are a synthetic MNIST-shaped draw, not MNIST"}
    else:
        r = model.result
        solves = r.solves
        if dist is not None:  # every rank's solve log (fit_rank returns this rank's only)
            allv = [None] * world_env
            dist.all_gather_object(allv, solves)
            solves = [s for v in allv for s in v]
        crit, crit_ms = critical_path(solves, a.topology)
        r0 = [s for s in solves if s["rank"] == 0]
        extra = {"n_sv": int(len(r.ids)), "rounds": r.rounds, "b": r.b, "converged": r.converged,
                 "sv_history": r.sv_history, "merged_history": r.merged_history,
                 "round_ms": [round(x, 3) for x in r.round_ms], "transport": r.transport,
                 "driver_train_ms": round(r.train_ms, 3), "rank0_phase_ms": r.phase_ms,
                 "per_round_critical_path": crit, "critical_path_solve_ms": crit_ms,
                 "critical_path_basis": "solo device time per solve (serial-solve rehearsal)"
                 if any(s.get("solo_ms", -1.0) >= 0 for s in solves) else "wall time per solve",
                 "row_cache_solves": int(sum(s.get("row_cache", False) for s in solves)),
                 "rank0_smo_iterations": int(sum(s["iterations"] for s in r0)),
                 "skipped_solves": int(sum(s["skipped"] for s in solves)),
                 "warmup_fit_ms": warm_ms,
                 "max_rank_smo_iterations": max(sum(s["iterations"] for s in solves if s["rank"] == q)
                                                for q in range(max(1, r.world))),
                 "note": "per_round_critical_path = [round, slowest local solve ms (tree: first layer), rank-0 "
                         "merge ms (tree: slowest rank of each later layer), their SMO iterations]; "
                         "the single-GPU trainer solves the same 60k problem in one 12,793-iteration SMO",
                 # recorded one-GPU rehearsal (solo-timed solves), not measured by this run: where the cascade
                 # overtakes one GPU -- partitions with resident Grams vs one SMO on the row cache
                 "large_n_crossover_rehearsal": {"n": 1000000, "star_p8_critical_path_s": 1.670,
                                                 "single_gpu_s": 2.072,
                                                 "source": "profiles/r2_largen_cascade_vs_1gpu.txt"}}
        if rank == 0:
            extra["accuracy"] = model.score(te.X, te.y)
        ref = (REF_STAR_S if a.topology == "star" else REF_TREE_S).get(a.gpus)
        if ref:
            extra["speedup_vs_ref_cascade_same_P"] = round(ref / value, 2)
        if a.baseline_1gpu > 0:  # the single-GPU trainer on this rank's GPU, same data, same process
            if dist is not None:
                dist.barrier()
            if rank == 0:
                full = tr if not multiproc else synthetic_mnist(a.n, seed=a.seed)
                full = full.compact() if a.input == "u8" else full
                SVC(device=str(dev), wss=a.wss).fit(full.X, full.y)  # warm
                ts = []
                for _ in range(a.baseline_1gpu):
                    sync()
                    tb = time.perf_counter()
                    SVC(device=str(dev), wss=a.wss).fit(full.X, full.y)
                    sync()
                    ts.append(time.perf_counter() - tb)
                one = float(np.median(ts))
                extra["single_gpu_s"] = round(one, 6)
                extra["speedup_vs_1gpu"] = round(one / value, 4)
            if dist is not None:
                dist.barrier()
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 6),
            "unit": "s",
            "n_gpus": a.gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": round(value / REF_GPU_S, 6),
            "dtype": "fp64",
            "data": "synthetic (deterministic MNIST-shaped 784-dim uint8 pixels, digit-1 one-vs-rest)",
            "config": {
                "model": f"RBF SVM, {a.wss}-order SMO (C=10, gamma=0.00125, tau=1e-5), MNIST-60k one-vs-rest",
                "global_batch": a.n,
                "seq_len": 784,
                "parallelism": "single-gpu" if not use_cascade else f"cascade-{a.topology}-dp{a.gpus}",
            },
            "launch": "torchrun (one rank per process)" if multiproc else
                      ("in-process thread ranks" if use_cascade else "single process"),
            **({"device": "cpu (C++ oracle; launch-path check, not a benchmark)"} if cpu else {}),
            "host_rows": "uint8 (widened to fp64 on device)" if a.input == "u8" else "fp64",
            "speedup_vs_serial": round(REF_SERIAL_S / value, 2),
            "speedup_vs_ref_gpu": round(REF_GPU_S / value, 2),
            "step_ms": step_ms,
            "step_upload_alloc_gram_smo_fit_ms": parts,
            **extra,
        }
        s = json.dumps(line)
        print(s, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(s + "\n")
    if crank is not None:
        crank.close()
    if group is not None:
        group.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
