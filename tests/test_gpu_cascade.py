"""Cascade SVM with the gfx950 device solver: multi-process SPMD ranks sharing one GPU (gloo group
for the exchanges, HIP for every solve), compared with the CPU-oracle cascade."""
import os
import socket

import numpy as np
import pytest
import torch

from svm355 import SVMParams
from svm355.parallel.cascade import CascadeSVM, partition_bounds
from svm355.parallel.transport import run_threads
from svm355.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu

N = 2000


def _worker(rank, world, port, topology, q):
    import torch.distributed as dist

    from svm355.parallel.transport import TorchDistTransport

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = synthetic_mnist(N, seed=21)
        te = synthetic_mnist(500, seed=21, offset=N)
        lo, hi = partition_bounds(N, world, rank)
        t = TorchDistTransport(torch.device("cpu"))
        c = CascadeSVM(t, SVMParams(), topology=topology, verbose=0, device=torch.device("cuda:0"))
        c.fit(tr.X[lo:hi], tr.y[lo:hi], np.arange(lo, hi), n_total=N)
        q.put((rank, c.summary(), c.score(te.X, te.y), sorted(c.result.sv.ids.tolist())))
    except BaseException as e:  # report instead of hanging the parent
        q.put((rank, {"error": repr(e)}, 0.0, []))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_multiprocess_hip_cascade_matches_cpu_cascade(topology):
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, topology, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=120)
    for _, s, _, _ in res:
        assert "error" not in s, s
    assert all(p.exitcode == 0 for p in procs)
    (_, s0, acc0, ids0), (_, s1, acc1, ids1) = res
    assert s0["converged"] and ids0 == ids1 and s0["b"] == s1["b"]

    tr = synthetic_mnist(N, seed=21)
    te = synthetic_mnist(500, seed=21, offset=N)

    def fn(t):
        lo, hi = partition_bounds(N, t.world, t.rank)
        c = CascadeSVM(t, SVMParams(n_threads=4), topology=topology, verbose=0)
        c.fit(tr.X[lo:hi], tr.y[lo:hi], np.arange(lo, hi), n_total=N)
        return c.summary(), c.score(te.X, te.y), sorted(c.result.sv.ids.tolist())

    cpu = run_threads(2, fn)[0]
    # Same cascade, kernel values differ in the last ulps (MFMA norm form vs direct sum).
    assert abs(s0["b"] - cpu[0]["b"]) < 1e-5 * max(1.0, abs(cpu[0]["b"]))
    assert len(set(ids0) ^ set(cpu[2])) <= 2
    assert abs(acc0 - cpu[1]) <= 0.002
