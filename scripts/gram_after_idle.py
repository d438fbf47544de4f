"""Does the Gram run slower after the device (or seven of its XCDs) idled?  Gram kernel time measured
with HIP events: back-to-back, after a host sleep, and right after an XCD-local SMO solve."""
import sys
import time

import torch

sys.path.insert(0, ".")
from svm355 import SVMParams  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

dev = torch.device("cuda:0")
n = 60000
tr = synthetic_mnist(n, seed=2024)
Xd = D.upload_rows(tr.compact().X, dev)
mn, mx, sqn = D.minmax_scale_(Xd, 784)
yd = torch.from_numpy(tr.y).to(dev)
K, _ = D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx)


def gram_ms():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    D.rbf_gram_sym(Xd, sqn, 0.00125, mn=mn, mx=mx, out=K)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


for label, before in (("back-to-back", lambda: None), ("after 50 ms host sleep", lambda: time.sleep(0.05)),
                      ("after 500 ms host sleep", lambda: time.sleep(0.5)),
                      ("after an XCD-local SMO", lambda: (D.smo(K, yd, torch.zeros(n, dtype=torch.float64, device=dev),
                                                              SVMParams(), n=n), torch.cuda.synchronize())),
                      ("back-to-back again", lambda: None)):
    v = []
    for _ in range(5):
        before()
        v.append(gram_ms())
    print(f"{label:26s}: " + " ".join(f"{x:.2f}" for x in v) + f"  (median {sorted(v)[2]:.2f} ms)", flush=True)
