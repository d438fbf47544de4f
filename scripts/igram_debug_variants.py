import os, sys, time, torch
sys.path.insert(0, ".")
from svm355.ops import device as D
from svm355.utils.data import synthetic_mnist
dev = torch.device("cuda:0"); n = 60000
tr = synthetic_mnist(n, seed=2024); Xd = D.upload_rows(tr.X, dev); mn, mx, sqn = D.minmax_scale_(Xd, 784)
K = torch.empty((n, n), dtype=torch.float64, device=dev)
for dbg in ("0", "1", "2", "3", "5", "7", "8", "15", "0"):
    os.environ["SVM355_IGRAM_DEBUG"] = dbg
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, gram="int", out=K)
        torch.cuda.synchronize(); best = min(best, time.perf_counter() - t0)
    print(f"dbg={dbg} (1 no mirror, 2 no exp, 4 no direct store, 8 no k-loop): {best*1e3:.2f} ms", flush=True)
