"""Is the first GPU operation after a fit slow?  Times a tiny torch copy and an RCCL barrier right
after (a) idle, (b) a single-GPU SVC fit, (c) a cascade fit."""
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355 import SVC, SVMParams  # noqa: E402
from svm355.parallel.cascade import CascadeSVM  # noqa: E402
from svm355.parallel.rccl import DeviceGroup, RcclRank  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
tr = synthetic_mnist(60000, seed=2024).compact()
small = synthetic_mnist(5000, seed=1).compact()
rank = RcclRank(0, RcclRank.unique_id(), 1, 0)
g = DeviceGroup(1, "rccl")
x = torch.zeros(1, device=dev)


def probe(tag):
    t0 = time.perf_counter()
    x.add_(1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    rank.barrier()
    t2 = time.perf_counter()
    rank.barrier()
    t3 = time.perf_counter()
    print(f"{tag:28s} torch op {1e3*(t1-t0):8.3f} ms | rccl barrier {1e3*(t2-t1):8.3f} ms | again {1e3*(t3-t2):7.3f} ms",
          flush=True)


for rep in range(3):
    probe("idle")
    SVC(device="cuda:0").fit(tr.X, tr.y)
    probe("after SVC 60k")
    SVC(device="cuda:0").fit(small.X, small.y)
    probe("after SVC 5k")
    CascadeSVM(SVMParams()).fit(tr.X, tr.y, world=1, device="cuda", group=g)
    probe("after cascade 60k")
    time.sleep(0.2)
    probe("after 200 ms sleep")
