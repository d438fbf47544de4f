"""One-vs-rest (all ten digits, the decomposition per class on concurrent host threads) at large n: ten
solver contexts share one GPU, each with its column cache; wall time, per-class stop reasons, accuracy."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from svm355.models.multiclass import OneVsRestSVC  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
tr = synthetic_mnist(n, seed=0).compact()
te = synthetic_mnist(5000, seed=0, offset=n).compact()
workers = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
for k, wk in enumerate(workers):
    torch.cuda.synchronize()
    t = time.perf_counter()
    m = OneVsRestSVC(device="cuda:0", max_iter=10_000_000, concurrent_solves=wk or None).fit(tr.X, tr.labels)
    torch.cuda.synchronize()
    w = time.perf_counter() - t
    reasons = sorted(set(m.stop_reasons_))
    ct = m.class_timings_
    print("  per class (solve ms / outer / pair updates):",
          "; ".join(f"{c}: {t['smo_ms']:.0f}/{t['outer_iterations']}/{t['inner_iterations']}" for c, t in sorted(ct.items())))
    print(f"fit {k}: concurrent_solves {wk or 'all'}: n={n} {w:.3f} s, accuracy {m.score(te.X, te.labels):.4f}, stop reasons {reasons}", flush=True)
