"""Where a cascade fit's wall time goes outside its solves: python call vs native group fit
(setup / ranks / output) vs the driver's own phases.  python scripts/cascade_overhead.py [P] [transport]"""
import os
import sys
import time

sys.path.insert(0, ".")
os.environ.setdefault("SVM355_CASCADE_PROFILE", "2")
from svm355 import SVMParams  # noqa: E402
from svm355.parallel.cascade import CascadeSVM  # noqa: E402
from svm355.parallel.rccl import DeviceGroup  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 1
transport = sys.argv[2] if len(sys.argv) > 2 else "auto"
tr = synthetic_mnist(60000, seed=2024).compact()
g = DeviceGroup(P, transport)
for rep in range(4):
    t0 = time.perf_counter()
    c = CascadeSVM(SVMParams()).fit(tr.X, tr.y, world=P, device="cuda", group=g)
    wall = (time.perf_counter() - t0) * 1e3
    r = c.result
    solve_ms = sum(s["ms"] for s in r.solves if s["rank"] == 0)
    gram_ms = sum(s["gram_ms"] for s in r.solves if s["rank"] == 0)
    print(f"P={P} rep {rep}: python wall {wall:.2f} ms | driver {r.train_ms:.2f} | rank0 solves {solve_ms:.2f} "
          f"(gram {gram_ms:.2f}) | phases {r.phase_ms}", flush=True)
g.close()
