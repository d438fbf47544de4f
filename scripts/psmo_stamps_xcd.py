"""Per-phase stamps of the persistent SMO, device-wide vs XCD-local, at one n."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
for n in [int(v) for v in (sys.argv[1:] or ["8700"])]:
    tr = synthetic_mnist(n, seed=2024)
    Xd = D.upload_rows(tr.X, dev)
    mn, mx, sqn = D.minmax_scale_(Xd, 784)
    K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)
    yd = torch.from_numpy(tr.y).to(dev)
    os.environ.update({"SVM355_SMO": "persistent", "SVM355_PSMO_STAMP": "1"})
    for xcd, nt in (("0", "512"), ("1", "256"), ("1", "512")):
        os.environ.update({"SVM355_PSMO_XCD": xcd, "SVM355_PSMO_NT": nt})
        print(f"n={n} xcd={xcd} NT={nt}", file=sys.stderr, flush=True)
        a = torch.zeros(n, dtype=torch.float64, device=dev)
        D.smo(K, yd, a, SVMParams(), n=n)
        torch.cuda.synchronize()
