"""Fixed cost of one cascade solve at cascade sizes (what a converged, 1-iteration solve costs).

For m rows of synthetic MNIST-shaped data, runs the cascade's HIP backend solve cold, then again
from the converged alphas (1 SMO iteration), and splits the warm solve into its host-visible
parts: row norms, y/alpha upload, Gram, warm f + SMO, alpha download, SV row gather."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.parallel.cascade import _HipBackend  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
P = SVMParams()
for m in [int(x) for x in (sys.argv[1:] or ["1380", "3500", "8700", "60000"])]:
    tr = synthetic_mnist(m, seed=2024).compact()
    be = _HipBackend(P, tr.X.shape[1], dev)
    X = be.to_rows(tr.X, dev)
    mn, mx = be.local_minmax(X)
    be.scale_(X, mn, mx)
    a0 = np.zeros(m)
    a, res = be.solve(X, tr.y, a0)
    cold_it = res.iterations
    D = be.D
    for rep in range(3):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        sqn = D.row_norms(X, be.d)
        torch.cuda.synchronize(); t.append(time.perf_counter())
        yd = torch.from_numpy(np.ascontiguousarray(tr.y, dtype=np.int32)).to(dev)
        ad = torch.from_numpy(a.copy()).to(dev)
        torch.cuda.synchronize(); t.append(time.perf_counter())
        r2, tm = D.train(X, sqn, yd, ad, P, warm=True, K=D.gram_buffer(m, dev), mn=be.stats[0], mx=be.stats[1])
        torch.cuda.synchronize(); t.append(time.perf_counter())
        ah = ad.cpu().numpy()
        t.append(time.perf_counter())
        keep = np.flatnonzero(ah > P.sv_tol)
        rows = be.select(X, keep)
        torch.cuda.synchronize(); t.append(time.perf_counter())
        d = [(t[i + 1] - t[i]) * 1e3 for i in range(len(t) - 1)]
    print(f"m={m:6d} cold it={cold_it:6d} | warm it={r2.iterations} total {sum(d):.3f} ms: norms {d[0]:.3f} "
          f"upload {d[1]:.3f} train {d[2]:.3f} (gram {tm['gram_ms']:.3f} smo {tm['smo_ms']:.3f} "
          f"lib total {tm['total_ms']:.3f}) alpha D2H {d[3]:.3f} gather {d[4]:.3f}  n_sv {len(keep)}", flush=True)
