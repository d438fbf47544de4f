"""Sequential per-class decomposition fits at 1M rows (one thread), free device memory before each, and the
solve time per outer iteration: does every class get its column cache?"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from svm355 import SVC  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import synthetic_mnist  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
release = len(sys.argv) > 2 and sys.argv[2] == "release"
tr = synthetic_mnist(n, seed=0).compact()
for c in range(10):
    y = np.where(tr.labels == c, 1, -1).astype(np.int32)
    free, total = torch.cuda.mem_get_info(0)
    t = time.perf_counter()
    m = SVC(device="cuda:0", solver="decomp", max_iter=10_000_000).fit(tr.X, y)
    torch.cuda.synchronize()
    w = time.perf_counter() - t
    tm = m.timings_
    import ctypes
    ctx = D.DeviceContext.get(torch.device("cuda:0"))
    slab = ctypes.c_int64(0)
    ctx.lib.svmd_cache_bytes(ctx.handle, None, ctypes.byref(slab))
    print(f"class {c}: free before {free / 2**30:.1f} GiB, fit {w:.3f} s, solve {tm['smo_ms']:.0f} ms, outer "
          f"{tm['outer_iterations']} ({tm['smo_ms'] / tm['outer_iterations']:.2f} ms each), slab after the fit {slab.value / 2**30:.1f} GiB", flush=True)
    if release:
        D.release_gram_buffers()
