"""Is the narrow column store's ~4 TB/s a property of its strided chunk reads?  The same int8 volume as
rows of one 128-byte chunk (d = 128: a 32-row tile is 4 KB contiguous, read by one chunk) against rows of
832 bytes (d = 832: seven 128-byte chunks per row, each chunk a strided 32 x 128-byte read).  Random uint8
rows (every column the full 0..255 range: one range group), m columns through the cache (kernel times by
rocprofv3)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from svm355.ops import device as D  # noqa: E402

dev = torch.device("cuda:0")
import os  # noqa: E402
os.environ["SVM355_GEMV_VIA_CACHE"] = "1"
for d, n in ((128, 6_500_000), (832, 1_000_000)):
    rng = np.random.default_rng(d)
    X = rng.integers(0, 256, size=(n, d), dtype=np.uint8)
    X[0], X[1] = 0, 255
    Xu = D.upload_u8(X, dev)
    del X
    mmd = torch.empty(2 * d, dtype=torch.float64, device=dev)
    D.minmax_u8(Xu, out=mmd)
    mm = mmd.cpu().numpy()
    cols = np.array([5], dtype=np.int32)
    for _ in range(10):
        D.decomp_gemv_u8(Xu, mm[:d].copy(), mm[d:].copy(), 1.0 / d, cols, np.ones(1))
    torch.cuda.synchronize()
    print(f"d={d} n={n}: {n * d / 1e6:.0f} MB of int8 rows, 10 one-column stores", flush=True)
    del Xu
    torch.cuda.empty_cache()
