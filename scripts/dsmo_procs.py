"""Per-process distributed SMO rehearsal on ONE GPU: `--world` processes (this script spawns them),
each one team on GPU 0; the receive arrays cross the processes as IPC handles (the torchrun form of
the 8-GPU run).  Every rank checks the result against the single-GPU solve."""
import argparse
import os
import subprocess
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=2)
ap.add_argument("--n", type=int, default=3000)
ap.add_argument("--child", type=int, default=-1)
ap.add_argument("--port", type=int, default=29631)
a = ap.parse_args()

if a.child < 0:
    procs = []
    for r in range(a.world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(a.world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port),
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-u", __file__, "--world", str(a.world), "--n", str(a.n),
                                       "--child", str(r)], env=env))
    rcs = [p.wait(timeout=120) for p in procs]
    print("child exit codes", rcs, flush=True)
    sys.exit(0 if all(rc == 0 for rc in rcs) else 1)

import datetime  # noqa: E402

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, ".")
from svm355 import SVC, SVMParams  # noqa: E402
from svm355.parallel.dsmo import DistributedSVC, DsmoRank  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
r = dist.get_rank()
tr = synthetic_mnist(a.n, seed=31).compact()
rk = DsmoRank.from_torch_dist(0, timeout_s=30)
print(f"rank {r}: connected", flush=True)
for rep in range(2):
    m = DistributedSVC(a.world, rank=rk).fit(tr.X, tr.y)
    ref = SVC(device="cuda:0").fit(tr.X, tr.y)
    same = m.n_iter_ == ref.n_iter_ and m.b_ == ref.b_ and np.array_equal(m.alpha_, ref.alpha_)
    print(f"rank {r} rep {rep}: {m.n_iter_} it b={m.b_!r} timings={m.timings_} identical={same}", flush=True)
    if not same:
        sys.exit(3)
rk.close()
dist.destroy_process_group()
