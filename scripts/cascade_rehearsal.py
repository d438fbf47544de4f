"""Cascade rehearsal on ONE GPU: P thread-ranks (ThreadTransport) share cuda:0, each with its own
device context/stream.  Reports the fit time and per-solve stats (n, iterations, ms) so the round
structure of the real P-GPU run can be read off (the per-rank solves of a round run concurrently
on the shared GPU, so absolute times are an upper bound for P separate GPUs)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.parallel.cascade import CascadeSVM, partition_bounds  # noqa: E402
from svm355.parallel.transport import run_threads  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
cfgs = sys.argv[2:] or ["star:1", "star:2", "star:4", "star:8", "tree:2", "tree:4", "tree:8"]
tr = synthetic_mnist(n, seed=2024)
te = synthetic_mnist(10000, seed=2024, offset=n)
dev = torch.device("cuda:0")
for cfg in cfgs:
    topo, P = cfg.split(":")
    P = int(P)

    def body(t):
        lo, hi = partition_bounds(n, P, t.rank)
        m = CascadeSVM(t, SVMParams(), topology=topo, verbose=0, device=dev)
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = m.fit(tr.X[lo:hi], tr.y[lo:hi], np.arange(lo, hi), n_total=n)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
        acc = m.score(te.X, te.y) if t.rank == 0 else None
        return dt, r, acc

    out = run_threads(P, body, lambda r: dev)
    dt, r, acc = out[0]
    print(f"{topo} P={P}: fit {dt:.1f} ms rounds {r.rounds} n_sv {len(r.sv)} b {r.b:.12f} acc {acc} "
          f"sv_history {r.sv_history} round_ms {[round(x, 1) for x in r.round_ms]}", flush=True)
    for o in out:
        for sv in o[1].solves:
            print(f"    r{sv['round']} rank{sv['rank']} {sv['layer']:>7}: n={sv['n']:6d} it={sv['iterations']:6d} "
                  f"{sv['ms']:7.2f} ms", flush=True)
