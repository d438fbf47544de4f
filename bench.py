#!/usr/bin/env python3
"""Headline benchmark: SMO train time on the MNIST-60k one-vs-rest RBF config (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 60000] [--parallel auto|smo|cascade]

One "step" is one complete training run on the fixed synthetic 60k x 784 MNIST-shaped matrix
(an SVM has no random init; the data are a deterministic synthetic draw of MNIST's shape and value
domain because MNIST itself is not available offline):

* N = 1: the single-GPU trainer (gpu_svm_main3.cu equivalent).  Timed scope = the reference's GPU
  "training" scope (gpu_svm_main3.cu:525-616): H2D of X and y, min/max + scaling, the kernel values,
  device SMO to convergence, SV extraction.  Rows are held as uint8 (what MNIST is) and quantised
  straight from the bytes, every kernel value exact in FP64 (``--input f64`` ships FP64 rows like the
  reference, same results).  ``--solver decomp`` (default): the SMO-type working-set decomposition
  solver (csrc/hip/decomp.hip) -- the reference's stop test b_low <= b_high + 2 tau on all n points
  and its clip / update arithmetic, reached through working sets of 1,024 points solved in one
  workgroup; same support-vector set as the pairwise solve, b within the reference's own
  serial-vs-GPU spread.  ``--solver smo``: the reference's pairwise first-order trajectory, bit for
  bit the CPU oracle's (resident exact-integer Gram + persistent device SMO); the JSON line reports
  the other solver's fit next to the headline either way.
* N > 1, ``--parallel auto`` with the decomposition solver (the default): the distributed
  decomposition solver (every GPU owns 1/N of the selection blocks and of f; one RCCL all-gather of
  candidate records per outer iteration); bit-identical to the one-GPU decomposition solver.  After
  it, on the same ranks and under the same bracket (max over ranks), the star and the tree cascade
  (BASELINE configs 5 and 4, every solve the warm-started decomposition): ``cascade_star_ms``,
  ``cascade_tree_ms`` and their rounds, SV history and critical path (``--cascade-steps``).
* N > 1, ``--parallel smo`` (``auto`` with ``--solver smo``): ONE first-order SMO over the N GPUs
  (csrc/hip/dsmo.hip): each GPU owns 1/N of the points and its slab K(:, own) of the exact-integer
  Gram, and the per-iteration arg-min / arg-max candidates cross the GPUs over xGMI -- the same
  problem, the same stop test and the same model as one GPU, bit for bit (strong scaling).
* N > 1, ``--parallel cascade`` (or ``--cascade``): the reference's multi-processor algorithm as the
  headline, the Cascade SVM (modified two-layer star, mpi_svm_main2.cpp, default; ``--topology tree``
  = classical mpi_svm_main3.cpp), one rank per GPU over RCCL; every local / merge solve is the
  warm-started decomposition (``--solver smo``: the reference's pairwise trajectory).  ``auto`` with
  ``--solver smo`` falls back to it when the distributed SMO is not applicable (non-pixel data) or its
  preflight fails.
Launch: directly (``python bench.py --gpus N``: N thread-ranks of this process, one GPU each) or by
torchrun (WORLD_SIZE = N: one rank per process on GPU LOCAL_RANK; the distributed SMO exchanges the
receive arrays' IPC handles, the cascade the ncclUniqueId, over the launcher's store).

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

# RCCL / IPC between processes (torchrun ranks) needs dmabuf IPC; the legacy IPC mode fails with
# "hipIpcGetMemHandle: invalid argument" on these hosts.  Must be set before the HSA runtime starts.
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

REF_GPU_S = 58.570  # GPU SMO training time, 60k
REF_SERIAL_S = 3285.662  # serial SMO training time, 60k
REF_GPU_PRED_S = 38.297  # GPU prediction time, 60k train / 10k test
REF_STAR_S = {4: 886.733, 8: 649.773, 16: 440.705, 32: 333.696, 64: 301.263}
REF_TREE_S = {4: 1194.269, 8: 839.406, 16: 662.153, 32: 671.448, 64: 673.580}
METRIC = "SMO train time (s) + speedup vs serial, MNIST-60k RBF; accuracy/#SV parity"


def ids_digest(ids) -> str:
    """Short digest of a support-vector id set (order-free), to compare SV sets across runs."""
    import hashlib

    return hashlib.sha1(np.sort(np.asarray(ids, dtype=np.int64)).tobytes()).hexdigest()[:16]
PREFLIGHT_ROWS = 4096


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    # --rows / --test-rows: spellings torchrun's own parser does not take for an abbreviation of its options
    ap.add_argument("--n", "--rows", dest="n", type=int, default=60000, help="training rows (MNIST-60k config)")
    ap.add_argument("--m", "--test-rows", dest="m", type=int, default=10000, help="test rows for the parity fields")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--parallel", choices=["auto", "smo", "cascade", "decomp"], default="auto",
                    help="N > 1: one distributed SMO over the GPUs (smo), the reference's Cascade SVM (cascade), "
                         "smo or the cascade, whichever fit is measured faster (auto), or the opt-in distributed "
                         "working-set decomposition solver (decomp; compared with the one-GPU decomposition solver)")
    ap.add_argument("--topology", choices=["star", "tree"], default="star")
    ap.add_argument("--transport", choices=["auto", "rccl", "loopback", "hostcomm"], default="auto",
                    help="direct launch, N > 1: one GPU per rank (auto / rccl), or loopback = a rehearsal of N ranks "
                         "on the visible GPU (cascade: host-staged exchanges; smo: N teams in one launch); under "
                         "torchrun: RCCL (auto / rccl) or hostcomm = the same per-process ranks exchanging over the "
                         "gloo group with host-staged device buffers, so N processes may share one GPU (the "
                         "per-process N-GPU path rehearsed on one device; decomp and cascade)")
    ap.add_argument("--allow-transport-fallback", action="store_true",
                    help="under torchrun: when the RCCL rank cannot be set up or fails its preflight on any rank, time "
                         "the same ranks over host-staged gloo exchanges (config.parallelism then ends in -gloo) "
                         "instead of exiting non-zero with the failing rank and step")
    ap.add_argument("--input", choices=["u8", "f64", "f64-real"], default="u8",
                    help="host row format: uint8 pixels (default), FP64 as in the reference, or f64-real: the same "
                         "rows plus a deterministic uniform [0, 0.5) offset per value (real-valued data: no "
                         "exact-integer plan, every kernel value on FP64 MFMA; --parallel decomp / cascade)")
    ap.add_argument("--cascade", action="store_true", help="run the cascade even with one GPU")
    ap.add_argument("--cascade-steps", type=int, default=2,
                    help="N > 1 with the distributed decomposition headline: the star and tree cascades (BASELINE "
                         "configs 5 / 4) are timed after it with this many fits each, same bracket and max over "
                         "ranks (0 = skip)")
    ap.add_argument("--baseline-1gpu", type=int, default=3,
                    help="N > 1: single-GPU fits timed after the run for speedup_vs_1gpu (0 = skip)")
    ap.add_argument("--wss", choices=["first", "second"], default="first",
                    help="working-set selection: first order (the reference; the headline) or the opt-in second-order")
    ap.add_argument("--solver", choices=["decomp", "smo"], default=None,
                    help="the working-set decomposition SMO (decomp; default on GPUs: same stop test on all n points, "
                         "same SVs; N > 1: --parallel auto runs it distributed) or the reference's pairwise first-order "
                         "trajectory (smo; the CPU oracle's, the default with --device cpu)")
    ap.add_argument("--max-iter", type=int, default=100000,
                    help="pair-update cap of every solve (the reference's 100,000; --rows beyond ~2M needs more)")
    ap.add_argument("--decomp-fits", "--other-solver-fits", dest="decomp_fits", type=int, default=3,
                    help="N = 1: fits of the OTHER solver (pairwise when the headline is decomp, and vice versa) timed "
                         "after the run and reported next to the headline (0 = skip)")
    ap.add_argument("--comm-timeout", type=float, default=120.0,
                    help="N > 1: seconds any rank waits on an exchange before every rank aborts its communicator "
                         "(a fit takes well under a second; a dead peer must not hang the run)")
    ap.add_argument("--f64-fits", type=int, default=3,
                    help="N = 1: steady-state fits with FP64 host rows (the reference's H2D), reported next to the "
                         "headline (0 = skip)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: the same launch paths on the C++ oracle (CPU tests of the torchrun / thread-rank "
                         "plumbing; N > 1 under torchrun exchanges over gloo); not a benchmark")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    a = ap.parse_args(argv)
    if a.steps < 1 or a.warmup < 0 or a.gpus < 1:
        ap.error("--steps must be >= 1, --warmup >= 0 and --gpus >= 1")

    import torch

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per process under torchrun; with one process (--cascade) the same per-process path runs
    # on a single GPU, so a one-GPU box rehearses the launch the N-GPU run takes
    multiproc = world_env > 1 or ("LOCAL_RANK" in os.environ and (a.cascade or a.parallel in ("smo", "decomp")))
    if multiproc and world_env != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        return 2
    cpu = a.device == "cpu"
    hostcomm = a.transport == "hostcomm"
    if hostcomm and not multiproc:
        print("bench.py: --transport hostcomm is a per-process transport (launch under torchrun)", file=sys.stderr)
        return 2
    cascade_solver = a.solver or "auto"  # the cascade's solves: per solve on GPUs unless --solver is given
    # the CPU oracle runs the pairwise SMO, except --parallel decomp: the decomposition's CPU twin
    cpu_smo = cpu and a.parallel != "decomp"
    if a.solver is None:  # the decomposition on GPUs (every cascade solve too); the pairwise SMO on the CPU oracle
        a.solver = "smo" if (cpu_smo or a.parallel == "smo") else "decomp"
    if a.solver == "decomp" and (cpu_smo or a.parallel == "smo"):
        print("bench.py: --solver decomp runs on GPUs (on the CPU only as --parallel decomp); the CPU oracle and the "
              "distributed pairwise SMO (--parallel smo) are --solver smo", file=sys.stderr)
        return 2
    ndev = torch.cuda.device_count() if not cpu else 1 << 30  # does not initialise the GPU on this image
    if not multiproc and a.gpus > 1 and a.transport != "loopback" and ndev < a.gpus:
        print(f"bench.py: --gpus {a.gpus} needs {a.gpus} visible GPUs, {ndev} visible "
              "(use --transport loopback for a one-GPU rehearsal)", file=sys.stderr)
        return 2
    if multiproc and ndev <= local_rank and not hostcomm:
        print(f"bench.py: LOCAL_RANK {local_rank} but {ndev} visible GPUs (--transport hostcomm lets processes share "
              "a GPU)", file=sys.stderr)
        return 2

    from svm355 import SVC, SVMParams
    from svm355.parallel.cascade import CascadeSVM, critical_path, partition_bounds
    from svm355.utils.data import synthetic_mnist

    dev_index = (local_rank % max(1, ndev) if hostcomm else local_rank) if multiproc else 0
    if not cpu:
        torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index) if not cpu else torch.device("cpu")
    sync = (lambda: torch.cuda.synchronize(dev)) if not cpu else (lambda: None)
    distributed = a.gpus > 1 or a.cascade or a.parallel in ("smo", "decomp")
    # A fresh process's first GPU operation (any: a copy, a PyTorch kernel, a context) pays a one-off
    # runtime/device initialisation (~85-115 ms, profiles/r3_first_op_probe.txt), whatever follows.
    # It is paid and timed here, outside the fits, so cold_fit_ms is the first fit's own cost.
    device_init_ms = None
    if not cpu:
        ti = time.perf_counter()
        torch.zeros(1, dtype=torch.uint8).to(dev)
        from svm355.ops import device as _D

        _D.DeviceContext.get(dev)
        sync()
        device_init_ms = round((time.perf_counter() - ti) * 1e3, 3)
    dist = None
    if multiproc:
        import torch.distributed as dist

        dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=10))  # bootstrap store + timing max

    params = SVMParams(wss=2 if a.wss == "second" else 1, max_iter=a.max_iter)
    te = synthetic_mnist(a.m, seed=a.seed, offset=a.n) if rank == 0 else None
    full = synthetic_mnist(a.n, seed=a.seed)  # every rank: the distributed SMO holds all rows on every GPU
    lo, hi = partition_bounds(a.n, world_env, rank) if multiproc else (0, a.n)
    part = full.subset(lo, hi)
    if a.input == "u8":
        full, part = full.compact(), part.compact()
        te = te.compact() if te is not None else None
    elif a.input == "f64-real":  # real-valued rows: the same pixels plus a fixed per-value offset in [0, 0.5)
        full.X = full.X + np.random.default_rng(a.seed + 7).uniform(0.0, 0.5, size=full.X.shape)
        part = full.subset(lo, hi)
        if te is not None:
            te.X = te.X + np.random.default_rng(a.seed + 8).uniform(0.0, 0.5, size=te.X.shape)
    pixel = full.X.dtype == np.uint8 and full.X.dtype == part.X.dtype

    mode = "single" if not distributed else ("cascade" if a.cascade else a.parallel)
    if mode == "auto" and a.solver == "decomp" and (pixel or a.input == "f64-real"):
        mode = "decomp"  # the headline solver, distributed (bit-identical to its one-GPU trajectory)
    auto = mode == "auto"
    fallback_reason = None
    if mode == "auto":
        mode = "smo" if (pixel and not cpu and a.wss == "first" and not a.cascade and a.gpus <= 8) else "cascade"
        if mode == "cascade":
            fallback_reason = ("not pixel rows" if not pixel else "cpu device" if cpu else "second-order selection"
                               if a.wss != "first" else "cascade requested" if a.cascade else "more than 8 GPUs")
    elif mode == "smo" and (cpu or not pixel) or mode == "decomp" and not cpu and not pixel and a.input != "f64-real":
        print(f"bench.py: --parallel {mode} needs uint8 pixel rows on GPUs (or --input f64-real for the "
              "decomposition's FP64 rows)", file=sys.stderr)
        return 2
    if hostcomm and mode not in ("decomp", "cascade"):
        print("bench.py: --transport hostcomm runs the per-process decomposition and cascade ranks", file=sys.stderr)
        return 2

    def agree(ok: bool) -> bool:
        """Every rank learns whether every rank succeeded (multi-process); the same bool otherwise."""
        if dist is None:
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    # ---- distributed SMO set-up + preflight: a 4096-row solve must equal the single-GPU solve
    group = crank = dgroup = drank = None
    # the exchanges' transport when it is not RCCL between GPUs: "gloo" (host-staged: --transport hostcomm, or the
    # opt-in fallback), "loopback" (a one-GPU rehearsal); the line's config.parallelism ends with it
    transport_label = "gloo" if hostcomm else "loopback" if a.transport == "loopback" else ""
    if mode == "smo":
        from svm355.parallel.dsmo import DistributedSVC, DsmoGroup, DsmoRank

        err = ""
        try:
            if multiproc:
                drank = DsmoRank.from_torch_dist(dev_index, timeout_s=a.comm_timeout)
            else:
                dgroup = DsmoGroup(a.gpus, rehearsal=a.transport == "loopback", timeout_s=a.comm_timeout)
        except Exception as e:  # noqa: BLE001 - reported, then the cascade runs
            err = f"set-up: {e}"
        if not agree(not err):
            fallback_reason = err or "set-up failed on another rank"
        else:
            pre = full.subset(0, min(PREFLIGHT_ROWS, a.n))
            try:
                m = DistributedSVC(a.gpus, group=dgroup, rank=drank, max_iter=a.max_iter).fit(pre.X, pre.y)
                ref = SVC(max_iter=a.max_iter, device=str(dev), solver="smo").fit(pre.X, pre.y)
                if not (m.n_iter_ == ref.n_iter_ and m.b_ == ref.b_ and np.array_equal(m.alpha_, ref.alpha_)):
                    err = (f"preflight differs from the single-GPU solve (iterations {m.n_iter_} vs {ref.n_iter_}, "
                           f"b {m.b_!r} vs {ref.b_!r})")
            except Exception as e:  # noqa: BLE001
                err = f"preflight: {e}"
            if not agree(not err):
                fallback_reason = err or "preflight failed on another rank"
        if fallback_reason:
            if rank == 0:
                print(f"bench.py: distributed SMO unavailable ({fallback_reason}); running the cascade",
                      file=sys.stderr, flush=True)
            mode = "cascade"
            for h in (dgroup, drank):
                if h is not None:
                    h.close()
            dgroup = drank = None

    def proc_rank():
        """This process's rank: gloo on the CPU oracle, host-staged gloo on the GPU, or RCCL."""
        if cpu:
            from svm355.parallel.hostcomm import HostCommRank

            return HostCommRank(comm_timeout_s=a.comm_timeout)
        if hostcomm:
            from svm355.parallel.hostcomm import HostCommDeviceRank

            return HostCommDeviceRank(dev_index, comm_timeout_s=a.comm_timeout)
        from svm355.parallel.rccl import RcclRank

        return RcclRank.from_torch_dist(dev_index, a.comm_timeout)

    if mode == "decomp":
        from svm355.parallel.decomp import DistributedDecompSVC

        if multiproc:
            # One rank per process.  Before any timed fit, a preflight solve of the first PREFLIGHT_ROWS rows
            # must equal the one-GPU solve bit for bit on every rank; if the RCCL rank cannot be set up or
            # its preflight fails on any rank, the ranks fall back together to the host-staged gloo
            # transport (the same driver; slower exchanges), and the line says why.
            err = ""
            try:
                crank = proc_rank()
            except Exception as e:  # noqa: BLE001 - the fallback below, reported in the line
                err = f"rank set-up: {type(e).__name__}: {e}"
            if agree(not err) and not cpu:
                pre = full.subset(0, min(PREFLIGHT_ROWS, a.n))
                try:
                    m = DistributedDecompSVC(a.gpus, rank=crank, max_iter=a.max_iter).fit(pre.X, pre.y)
                    ref = SVC(max_iter=a.max_iter, device=str(dev), solver="decomp").fit(pre.X, pre.y)
                    if 8 % a.gpus == 0:  # the one-GPU block partition: the same trajectory bit for bit
                        same = m.n_iter_ == ref.n_iter_ and m.b_ == ref.b_ and np.array_equal(m.alpha_, ref.alpha_)
                    else:  # another partition (a multiple of 8 x world blocks): another path to the same optimum
                        same = (m.stop_reason_ == ref.stop_reason_ == "converged" and abs(m.b_ - ref.b_) <= 10 * ref.params.tau
                                and abs(len(m.support_) - len(ref.support_)) <= max(2, len(ref.support_) // 100))
                    if not same:
                        err = (f"preflight differs from the one-GPU solve (iterations {m.n_iter_} vs {ref.n_iter_}, "
                               f"b {m.b_!r} vs {ref.b_!r})")
                except Exception as e:  # noqa: BLE001
                    err = f"preflight: {type(e).__name__}: {e}"
            if not agree(not err):
                if cpu or hostcomm:
                    print(f"bench.py rank {rank}: distributed decomposition unavailable: {err or 'another rank'}",
                          file=sys.stderr, flush=True)
                    os._exit(1)
                errs = [None] * world_env  # every rank's reason, so the line names the failing rank and step
                dist.all_gather_object(errs, err)
                failed = "; ".join(f"rank {r}: {e}" for r, e in enumerate(errs) if e)
                if not a.allow_transport_fallback:
                    if rank == 0:
                        print(f"bench.py: the RCCL transport failed ({failed}); not timing another transport under "
                              "the RCCL label (--allow-transport-fallback times host-staged gloo exchanges, labelled "
                              "-gloo)", file=sys.stderr, flush=True)
                    os._exit(1)
                transport_label = "gloo"
                fallback_reason = f"RCCL: {failed}; exchanges over gloo (host-staged)"
                if rank == 0:
                    print(f"bench.py: {fallback_reason}", file=sys.stderr, flush=True)
                if crank is not None:
                    try:
                        crank.close()
                    except Exception:  # noqa: BLE001 - an aborted communicator
                        pass
                from svm355.parallel.hostcomm import HostCommDeviceRank

                crank = HostCommDeviceRank(dev_index, comm_timeout_s=a.comm_timeout)
        elif cpu:
            pass  # thread ranks on the CPU oracle (DistributedDecompSVC(transport="cpu"))
        else:
            from svm355.parallel.rccl import DeviceGroup

            group = DeviceGroup(a.gpus, a.transport, a.comm_timeout)

    # auto with both applicable: the cascade is set up too and the faster measured fit runs (below)
    if mode == "cascade" or (auto and mode == "smo"):
        if multiproc:
            crank = proc_rank()
        elif not cpu:
            from svm355.parallel.rccl import DeviceGroup

            group = DeviceGroup(a.gpus, a.transport, a.comm_timeout)

    cascade_comm_ok = [True]  # false once a failed cascade aborted the ranks' communicators

    def barrier_sync():
        sync()
        if crank is not None and cascade_comm_ok[0]:
            crank.barrier()  # RCCL all-reduce over the cascade's own communicators
        if dist is not None:
            dist.barrier()
        sync()

    model = None

    def step():
        nonlocal model
        if mode == "single":
            model = SVC(max_iter=a.max_iter, device=str(dev), wss=a.wss, solver=a.solver).fit(full.X, full.y)
        elif mode == "smo":
            model = DistributedSVC(a.gpus, group=dgroup, rank=drank, max_iter=a.max_iter).fit(full.X, full.y)
        elif mode == "decomp":
            model = DistributedDecompSVC(a.gpus, group=group, rank=crank, max_iter=a.max_iter,
                                         transport="cpu" if cpu else "auto").fit(full.X, full.y)
        else:
            model = cascade_fit(a.topology)

    # fault injection (tests): SVM355_BENCH_CASCADE_FAIL="rank,round" makes that cascade rank fail at that round
    cfail = [int(v) for v in os.environ.get("SVM355_BENCH_CASCADE_FAIL", "-1,-1").split(",")]

    def cascade_fit(topology):
        c = CascadeSVM(params, topology=topology, comm_timeout_s=a.comm_timeout, solver=cascade_solver,
                       fail_rank=cfail[0], fail_round=cfail[1])
        if multiproc:
            return c.fit_rank(crank, part.X, part.y, np.arange(lo, hi), a.n)
        return c.fit(full.X, full.y, world=a.gpus, device="cpu" if cpu else "cuda", group=group)

    def guarded_step():
        try:
            step()
        except Exception as e:  # noqa: BLE001
            if multiproc:  # an orderly exit would wait for the process group's teardown on the peers
                print(f"bench.py rank {rank}: {mode} fit failed: {e}", file=sys.stderr, flush=True)
                os._exit(1)
            raise

    auto_selection = None
    if auto and mode == "smo":
        # Both N-GPU trainers apply: time one warm fit of each (bracketed like the timed steps, max
        # over ranks) and run the faster.  The distributed SMO's model is the single-GPU trainer's;
        # the cascade's is the reference's multi-processor algorithm.
        def once():
            guarded_step()  # warm
            barrier_sync()
            tt = time.perf_counter()
            guarded_step()
            barrier_sync()
            dt = torch.tensor([time.perf_counter() - tt], dtype=torch.float64)
            if dist is not None:
                dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            return float(dt.item()) * 1e3

        t_smo = once()
        mode = "cascade"
        t_casc = once()
        mode = "smo" if t_smo <= t_casc else "cascade"
        auto_selection = {"smo_fit_ms": round(t_smo, 3), "cascade_fit_ms": round(t_casc, 3), "chosen": mode}
        if mode == "smo":
            for h in (crank, group):
                if h is not None:
                    h.close()
            crank = group = None
        else:
            for h in (dgroup, drank):
                if h is not None:
                    h.close()
            dgroup = drank = None
            fallback_reason = "the cascade's measured fit was faster"

    warm_ms = []
    for _ in range(a.warmup):
        tw = time.perf_counter()
        guarded_step()
        sync()
        warm_ms.append(round((time.perf_counter() - tw) * 1e3, 3))
    barrier_sync()
    t0 = time.perf_counter()
    marks, parts = [], []
    for _ in range(a.steps):
        guarded_step()
        marks.append(time.perf_counter())  # host-side step boundaries (diagnostic only)
        if mode == "single":  # per-step upload / Gram / SMO split (diagnostic only)
            parts.append([round(model.timings_.get(k, 0.0), 2) for k in ("upload_preprocess_ms", "gram_alloc_ms",
                                                                           "gram_ms", "smo_ms")]
                         + [round(model.fit_time_ * 1e3, 2)])
        elif mode == "smo":
            t = model.timings_
            parts.append([round(t["upload_minmax_ms"], 2), round(t["quantise_slab_ms"], 2), round(t["smo_ms"], 2),
                          round(model.fit_time_ * 1e3, 2)])
    barrier_sync()
    elapsed = time.perf_counter() - t0
    step_ms = [round((b - a_) * 1e3, 3) for a_, b in zip([t0] + marks[:-1], marks)]
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    ms = elapsed / a.steps * 1e3
    value = ms / 1e3

    # BASELINE configs 5 / 4 (the reference's multi-processor programs, mpi_svm_main2.cpp star and
    # mpi_svm_main3.cpp tree) on the same ranks after the headline: each timed like the headline steps
    # (barrier + device sync on both sides, max over ranks), with its rounds, SV history and critical path.
    cascades = {}
    if mode == "decomp" and a.cascade_steps > 0 and not cpu:
        # After the headline: a cascade that fails (on any rank) is reported in the line instead of ending
        # the run -- the headline was already measured.  Its ranks' communicators are then aborted, so no
        # further cascade runs and the closing barriers skip them (the launcher's gloo group still works).
        for topo in ("star", "tree"):
            if topo == "tree" and a.gpus & (a.gpus - 1):
                cascades[f"cascade_{topo}"] = {"skipped": "the classical cascade needs a power-of-2 number of GPUs"}
                continue

            def run_topo():
                cm = cascade_fit(topo)  # warm
                barrier_sync()
                tc = time.perf_counter()
                for _ in range(a.cascade_steps):
                    cm = cascade_fit(topo)
                barrier_sync()
                return cm, (time.perf_counter() - tc) / a.cascade_steps

            err = ""
            try:
                cm, cel = run_topo()
            except Exception as e:  # noqa: BLE001 - reported in the JSON line
                err = f"{type(e).__name__}: {e}"
                print(f"bench.py rank {rank}: cascade ({topo}) failed: {err}", file=sys.stderr, flush=True)
            if not agree(not err):
                cascades[f"cascade_{topo}"] = {"error": err or "failed on another rank"}
                cascade_comm_ok[0] = False
                break
            if dist is not None:
                e = torch.tensor([cel], dtype=torch.float64)
                dist.all_reduce(e, op=dist.ReduceOp.MAX)
                cel = float(e.item())
            r = cm.result
            solves = r.solves
            if dist is not None:
                allv = [None] * world_env
                dist.all_gather_object(allv, solves)
                solves = [s for v in allv for s in v]
            crit, crit_ms = critical_path(solves, topo)
            ref = (REF_STAR_S if topo == "star" else REF_TREE_S).get(a.gpus)
            rec = {"ms": round(cel * 1e3, 3), "steps": a.cascade_steps, "rounds": r.rounds, "converged": r.converged,
                   "n_sv": int(len(r.ids)), "sv_ids_digest": ids_digest(r.ids), "b": r.b,
                   "sv_history": r.sv_history, "solver": cm.solver_used,
                   "transport": r.transport, "per_round_critical_path": crit, "critical_path_solve_ms": crit_ms,
                   "speedup_vs_ref_cascade_same_P": round(ref / cel, 2) if ref and a.n == 60000 else None,
                   "speedup_vs_serial": round(REF_SERIAL_S / cel, 2) if a.n == 60000 else None,
                   "b_minus_headline_b": float(r.b - model.b_)}
            if topo == "star":
                rec["merged_history"] = r.merged_history
            if rank == 0:
                rec["accuracy"] = cm.score(te.X, te.y)
            cascades[f"cascade_{topo}_ms"] = rec["ms"]
            cascades[f"cascade_{topo}"] = rec
    extra = {}
    if mode == "single":
        # Prediction on the 10k test rows (outside the timed region): H2D, scaling with the training
        # statistics, MFMA cross-kernel against the SVs, decision values back to the host.  The
        # reference's GPU "prediction" (38.3 s at 60k) also parses the test CSV.
        sync()
        tp = time.perf_counter()
        model.decision_function(te.X)
        sync()
        pred_ms = (time.perf_counter() - tp) * 1e3
        acc = model.score(te.X, te.y)
        f64_ms = []
        if a.f64_fits > 0 and not cpu and a.input == "u8":  # the reference's FP64 host rows, same model
            X64 = full.X.astype(np.float64)
            m64 = SVC(max_iter=a.max_iter, device=str(dev), wss=a.wss, solver=a.solver).fit(X64, full.y)
            for _ in range(a.f64_fits):
                sync()
                tf = time.perf_counter()
                m64 = SVC(max_iter=a.max_iter, device=str(dev), wss=a.wss, solver=a.solver).fit(X64, full.y)
                sync()
                f64_ms.append((time.perf_counter() - tf) * 1e3)
            extra["f64_input_fit_ms"] = round(float(np.median(f64_ms)), 3)
            extra["f64_input_same_model"] = bool(m64.b_ == model.b_ and m64.n_iter_ == model.n_iter_ and
                                                 np.array_equal(m64.alpha_, model.alpha_))
        other = "smo" if a.solver == "decomp" else "decomp"
        if a.decomp_fits > 0 and not cpu and a.input == "u8" and other == "smo" and a.n > 1048576:
            # beyond the pairwise solver's HBM row cache its fit replays kernels per iteration (minutes)
            extra["pairwise_solver"] = {"skipped": "n beyond the pairwise row cache (1,048,576 rows)"}
        elif a.decomp_fits > 0 and not cpu and a.input == "u8":
            # the other solver on the same rows (outside the timed region): the same stop test on all n
            # points by a different pair sequence; the same SV set expected, b within a few tau
            dm = SVC(max_iter=a.max_iter, device=str(dev), solver=other).fit(full.X, full.y)
            d_ms = []
            for _ in range(a.decomp_fits):
                sync()
                tf = time.perf_counter()
                dm = SVC(max_iter=a.max_iter, device=str(dev), solver=other).fit(full.X, full.y)
                sync()
                d_ms.append((time.perf_counter() - tf) * 1e3)
            rec = {"fit_ms": round(float(np.median(d_ms)), 3), "fit_ms_all": [round(x, 3) for x in d_ms],
                   "same_svs": bool(np.array_equal(dm.support_, model.support_)), "b": float(dm.b_),
                   "b_minus_headline_b": float(dm.b_ - model.b_), "iterations": int(dm.n_iter_),
                   "accuracy": dm.score(te.X, te.y), "stop_reason": dm.stop_reason_}
            if other == "decomp":
                rec.update(outer_iterations=dm.timings_["outer_iterations"], working_set=dm.timings_["working_set"])
                extra["decomp_solver"] = rec
            else:
                rec.update(timings_ms=dm.timings_, trajectory="the reference's pairwise first-order SMO, bit-identical "
                                                              "to the CPU oracle (tests/test_gpu_kernels.py)")
                extra["pairwise_solver"] = rec
        extra.update({
            "n_sv": int(len(model.support_)), "iterations": int(model.n_iter_), "b": float(model.b_),
            "accuracy": acc, "stop_reason": model.stop_reason_, "timings_ms": model.timings_,
            "prediction_ms_10k": round(pred_ms, 3), "ref_gpu_prediction_s": REF_GPU_PRED_S,
            "cold_fit_ms": warm_ms[0] if warm_ms else None, "warmup_fit_ms": warm_ms,
            "device_init_ms": device_init_ms, "solver": a.solver,
            "caveats": "timed fits reuse the library's grow-only device buffers and device context, allocated by the "
                       "first (cold) fit, whose time is cold_fit_ms (measured after the process's one-off device "
                       "initialisation, device_init_ms, which its first GPU operation of any kind pays); host rows are "
                       "uint8 pixels: min/max and the exact-integer quantisation read the bytes on the device and only "
                       "the support vectors are widened to scaled fp64 (f64_input_fit_ms: the same fit from the "
                       "reference's fp64 host rows); the data are a synthetic MNIST-shaped draw, not MNIST" +
                       ("; solver = the SMO-type working-set decomposition: the reference's stop test on all n points "
                        "and clip/update arithmetic, a different pair sequence than the reference's pairwise solve "
                        "(pairwise_solver: that solve's fit, SV set and b on the same rows)"
                        if a.solver == "decomp" else "")})
    elif mode == "decomp":
        extra = {"n_sv": int(len(model.support_)), "fallback_reason": fallback_reason, "iterations": int(model.n_iter_), "b": float(model.b_),
                 "stop_reason": model.stop_reason_, "decomp_stats": model.stats_, "rank_ms": model.rank_ms_,
                 "rank_host_wait_ms": getattr(model, "host_wait_ms_", None),
                 "warmup_fit_ms": warm_ms, "cold_fit_ms": warm_ms[0] if warm_ms else None,
                 "launch_form": ("one rank per process" + (" (CPU oracle over gloo)" if cpu else
                                                           f" over gloo, host-staged ({a.gpus} processes on "
                                                           f"{min(ndev, a.gpus)} GPU(s))"
                                                           if type(crank).__name__ == "HostCommDeviceRank" else " (RCCL)")
                                 if multiproc else "thread ranks on the CPU oracle (loopback)" if cpu
                                 else "thread ranks, one GPU each")
                 if a.transport != "loopback" else f"rehearsal: {a.gpus} ranks on one GPU",
                 "note": "working-set decomposition solver over all GPUs: every GPU holds all rows and an "
                         "alpha replica, owns 1/N of the selection blocks and of f, and all-gathers its candidate "
                         "records once per outer iteration; the working-set solve is replicated.  Compared with "
                         "the one-GPU decomposition solver (single_gpu_s, bit_identical_to_1gpu)"}
        if rank == 0:
            extra["accuracy"] = model.score(te.X, te.y)
    elif mode == "smo":
        extra = {"n_sv": int(len(model.support_)), "iterations": int(model.n_iter_), "b": float(model.b_),
                 "stop_reason": model.stop_reason_, "timings_ms": model.timings_, "team_shape": model.shape_,
                 "warmup_fit_ms": warm_ms, "cold_fit_ms": warm_ms[0] if warm_ms else None,
                 "launch_form": "one team per GPU" if a.transport != "loopback" else
                                f"rehearsal: {a.gpus} teams on one GPU",
                 "note": "one first-order SMO over all GPUs: each GPU holds 1/N of the points and its slab K(:, own) "
                         "of the exact-integer Gram; every iteration's candidates cross the GPUs over xGMI; same "
                         "iterations, alphas and b as the single-GPU trainer (bit_identical_to_1gpu)"}
        if rank == 0:
            extra["accuracy"] = model.score(te.X, te.y)
    else:
        r = model.result
        solves = r.solves
        if dist is not None:  # every rank's solve log (fit_rank returns this rank's only)
            allv = [None] * world_env
            dist.all_gather_object(allv, solves)
            solves = [s for v in allv for s in v]
        crit, crit_ms = critical_path(solves, a.topology)
        r0 = [s for s in solves if s["rank"] == 0]
        extra = {"n_sv": int(len(r.ids)), "sv_ids_digest": ids_digest(r.ids), "solver": model.solver_used,
                 "rounds": r.rounds, "b": r.b, "converged": r.converged,
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
                         "the single-GPU trainer solves the same 60k problem in one 12,793-iteration SMO"}
        if rank == 0:
            extra["accuracy"] = model.score(te.X, te.y)
        ref = (REF_STAR_S if a.topology == "star" else REF_TREE_S).get(a.gpus)
        if ref:
            extra["speedup_vs_ref_cascade_same_P"] = round(ref / value, 2)
        if fallback_reason:
            extra["fallback_reason"] = fallback_reason
    if mode in ("smo", "cascade", "decomp") and a.baseline_1gpu > 0:  # the single-GPU trainer, rank 0's GPU
        if dist is not None:
            dist.barrier()
        if rank == 0:
            one_solver = a.solver if mode in ("decomp", "cascade") else "smo"

            def one_fit():
                if cpu and mode == "decomp":  # the one-rank CPU oracle of the decomposition
                    return DistributedDecompSVC(1, transport="cpu", max_iter=a.max_iter).fit(full.X, full.y)
                return SVC(max_iter=a.max_iter, device=str(dev), wss=a.wss, solver=one_solver).fit(full.X, full.y)

            one = one_fit()  # warm
            ts = []
            for _ in range(a.baseline_1gpu):
                sync()
                tb = time.perf_counter()
                one = one_fit()
                sync()
                ts.append(time.perf_counter() - tb)
            t1 = float(np.median(ts))
            extra["single_gpu_s"] = round(t1, 6)
            extra["speedup_vs_1gpu"] = round(t1 / value, 4)
            if mode in ("smo", "decomp"):
                extra["bit_identical_to_1gpu"] = bool(one.n_iter_ == model.n_iter_ and one.b_ == model.b_ and
                                                      np.array_equal(one.alpha_, model.alpha_))
                if mode == "decomp" and 8 % a.gpus:  # a block partition of 8 x world blocks: another trajectory
                    extra["bit_identity_expected"] = False
                    extra["b_minus_1gpu_b"] = float(model.b_ - one.b_)
        if dist is not None:
            dist.barrier()
    if auto_selection is not None:
        extra["auto_selection"] = auto_selection
    extra.update(cascades)
    if distributed and not cpu:
        try:
            from svm355.parallel.rccl import rccl_info

            extra.update(rccl_info())
        except Exception as e:  # noqa: BLE001 - informative only
            extra["rccl_info_error"] = str(e)
    if rank == 0:
        if mode == "single":
            parallelism = "single-gpu"
        elif mode == "smo":
            parallelism = f"distributed-smo-dp{a.gpus}" + (f"-{transport_label}" if transport_label else "")
        elif mode == "decomp":
            parallelism = f"distributed-decomp-dp{a.gpus}" + (f"-{transport_label}" if transport_label else "")
        else:
            parallelism = f"cascade-{a.topology}-dp{a.gpus}" + (f"-{transport_label}" if transport_label else "")
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
            "vs_baseline": round(value / REF_GPU_S, 6) if a.n == 60000 else None,  # the reference's 60k time
            "dtype": "fp64",
            "data": ("synthetic (deterministic MNIST-shaped 784-dim uint8 pixels, digit-1 one-vs-rest)"
                     if a.input != "f64-real" else "synthetic (MNIST-shaped 784-dim pixels plus a uniform [0, 0.5) "
                     "offset per value: real-valued FP64 rows, digit-1 one-vs-rest)"),
            "config": {
                "model": (f"RBF SVM, {a.wss}-order SMO" if a.solver == "smo" and mode != "decomp"
                          else "RBF SVM, SMO-type working-set decomposition (reference stop test on all n points)")
                         + " (C=10, gamma=0.00125, tau=1e-5), "
                         + ("MNIST-60k one-vs-rest" if a.n == 60000 else f"MNIST-shaped one-vs-rest, {a.n:,} rows"),
                "global_batch": a.n,
                "seq_len": 784,
                "parallelism": parallelism,
            },
            "launch": "torchrun (one rank per process)" if multiproc else
                      ("in-process thread ranks" if distributed else "single process"),
            **({"device": "cpu (C++ oracle; launch-path check, not a benchmark)"} if cpu else {}),
            "host_rows": "uint8 (the device reads the bytes; only the SVs are widened to fp64)" if a.input == "u8"
                         else "fp64 (real-valued)" if a.input == "f64-real"
                         else "fp64",
            "speedup_vs_serial": round(REF_SERIAL_S / value, 2) if a.n == 60000 else None,
            "speedup_vs_ref_gpu": round(REF_GPU_S / value, 2) if a.n == 60000 else None,
            "step_ms": step_ms,
            ("step_upload_alloc_gram_smo_fit_ms" if mode != "smo" else "step_upload_slab_smo_fit_ms"): parts,
            **extra,
        }
        s = json.dumps(line)
        print(s, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(s + "\n")
    for h in (crank, group, dgroup, drank):
        if h is not None:
            try:
                h.close()
            except Exception as e:  # noqa: BLE001 - an aborted communicator; the line is already printed
                print(f"bench.py rank {rank}: close: {e}", file=sys.stderr, flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
