#!/usr/bin/env python3
"""The Newton polish step (decomp_newton.h) alone on the device against its host reference: a working set
of m synthetic-MNIST points (the solver's RBF, gamma 0.00125) with nf of them free, the rest at 0.
Prints bit-identity with the reference, the step's code, the mean time per step and its phases."""
import sys

import numpy as np

sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
from svm355 import _native as N  # noqa: E402
from svm355.ops import device as D  # noqa: E402
from svm355.utils.data import MinMaxScaler, synthetic_mnist  # noqa: E402

for m, nf in [(700, 339), (1024, 500), (400, 100)]:
    tr = synthetic_mnist(m, seed=7)
    X = MinMaxScaler().fit_transform(tr.X)
    sq = (X * X).sum(1)
    K = np.exp(-0.00125 * np.maximum(sq[:, None] + sq[None, :] - 2 * X @ X.T, 0.0))
    np.fill_diagonal(K, 1.0)
    y = tr.y.astype(np.int32)
    rng = np.random.default_rng(m)
    a = np.zeros(m)
    free = rng.choice(m, size=nf, replace=False)
    a[free] = rng.uniform(0.5, 9.5, size=nf)
    yp, yn = free[y[free] == 1], free[y[free] == -1]
    a[yp] *= a[yn].sum() / a[yp].sum()  # sum y a = 0
    f = K @ (a * y) - y
    ar, fr, cr = N.newton_step_probe(K, y, a, f, C=10.0)
    ad, fd, cd, prof, ms = D.decomp_newton_probe(K, y, a, f, C=10.0, reps=5)
    ph = np.diff(np.r_[prof[7], prof[:6]]) / 100.0  # 100 MHz ticks -> us
    print(f"m={m} nf={int(prof[6])}: code {cd} (ref {cr})  alpha bit-identical {np.array_equal(ad, ar)}  "
          f"f bit-identical {np.array_equal(fd, fr)}  {ms * 1e3:.1f} us/step  phases us: free {ph[0]:.1f} "
          f"K_FF {ph[1]:.1f} chol {ph[2]:.1f} (row updates {prof[8] / 100:.1f} block {prof[9] / 100:.1f} "
          f"solve+store {prof[10] / 100:.1f} staging {prof[11] / 100:.1f}) backsub {ph[3]:.1f} step {ph[4]:.1f} "
          f"f {ph[5]:.1f}", flush=True)
