import os, socket, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams
from svm355.parallel.cascade import CascadeSVM, partition_bounds
from svm355.utils.data import synthetic_mnist, MinMaxScaler
from svm355.ops import cpu as C

def worker(rank, world, port):
    import torch.distributed as dist
    from svm355.parallel.transport import TorchDistTransport
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N = 2000
    tr = synthetic_mnist(N, seed=21); te = synthetic_mnist(500, seed=21, offset=N)
    lo, hi = partition_bounds(N, world, rank)
    t = TorchDistTransport(torch.device("cpu"))
    c = CascadeSVM(t, SVMParams(), topology="star", verbose=0, device=torch.device("cuda:0"))
    c.fit(tr.X[lo:hi], tr.y[lo:hi], np.arange(lo, hi), n_total=N)
    r = c.result
    dec = c.decision_function(te.X)
    sc = MinMaxScaler(r.mn.cpu().numpy(), r.mx.cpu().numpy())
    svX = r.sv.X[:, :784].cpu().numpy()
    ref = C.decision(svX, r.sv.y, r.sv.alpha, sc.transform(te.X), 0.00125, r.b)
    ref2 = C.decision(sc.transform(tr.X[r.sv.ids]), r.sv.y, r.sv.alpha, sc.transform(te.X), 0.00125, r.b)
    if rank == 0:
        print("nsv", len(r.sv), "b", r.b, "dec[:5]", dec[:5], "ref[:5]", ref[:5], "ref2[:5]", ref2[:5], flush=True)
        print("max|dec-ref|", np.abs(dec-ref).max(), "max|ref-ref2|", np.abs(ref-ref2).max(), "acc", c.score(te.X, te.y), flush=True)
        print("mn", r.mn[:5].cpu().numpy(), "mx", r.mx[100:105].cpu().numpy(), "svX sum", svX.sum(), "true", sc.transform(tr.X[r.sv.ids]).sum(), flush=True)
    dist.destroy_process_group()

if __name__ == "__main__":
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]
    mp.start_processes(worker, args=(2, port), nprocs=2, start_method="spawn")
