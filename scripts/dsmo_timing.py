"""Timing of the distributed SMO rehearsal (P teams on one GPU) against the single-GPU trainer at n."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from svm355 import SVC, SVMParams  # noqa: E402
from svm355.parallel.dsmo import DsmoGroup  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

ns = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "60000").split(",")]
Ps = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4,8").split(",")]
for n in ns:
    tr = synthetic_mnist(n, seed=2024).compact()
    SVC(device="cuda:0").fit(tr.X, tr.y)
    ts = []
    for _ in range(3):
        m = SVC(device="cuda:0").fit(tr.X, tr.y)
        ts.append(m.fit_time_ * 1e3)
    print(f"n={n} single GPU: fit {np.median(ts):.2f} ms, smo {m.timings_['smo_ms']:.2f} ms, "
          f"{m.n_iter_} it, {m.timings_['smo_ms'] * 1e3 / m.n_iter_:.3f} us/it, b={m.b_!r}", flush=True)
    for P in Ps:
        g = DsmoGroup(P, rehearsal=True)
        g.fit(tr.X, tr.y)
        rows = []
        for _ in range(3):
            t0 = time.perf_counter()
            out = g.fit(tr.X, tr.y)
            rows.append(((time.perf_counter() - t0) * 1e3, out))
        rows.sort(key=lambda r: r[0])
        wall, out = rows[1]
        tm = out["timings_ms"]
        print(f"n={n} dsmo rehearsal P={P}: fit {wall:.2f} ms | upload+minmax {tm['upload_minmax_ms']:.2f} "
              f"quantise+slabs {tm['quantise_slab_ms']:.2f} smo {tm['smo_ms']:.2f} ms | {out['iterations']} it, "
              f"{tm['smo_ms'] * 1e3 / out['iterations']:.3f} us/it | b={out['b']!r} same={out['b'] == m.b_} "
              f"shape={out['shape']}", flush=True)
        g.close()
