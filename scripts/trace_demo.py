#!/usr/bin/env python3
"""The Python-side roctx ranges (svm355/utils/trace.py) around real work, for a marker trace:

    rocprofv3 --marker-trace --kernel-trace --output-format csv -d out -o run -- python3 scripts/trace_demo.py

a distributed decomposition fit (2 loopback ranks), a star cascade (per-solve solver) and a one-vs-rest
fit on synthetic MNIST."""
import numpy as np

from svm355.models.multiclass import OneVsRestSVC
from svm355.parallel.cascade import CascadeSVM
from svm355.parallel.decomp import DistributedDecompSVC
from svm355.utils.data import synthetic_mnist

tr = synthetic_mnist(20000, seed=3).compact()
m = DistributedDecompSVC(world=2, transport="loopback").fit(tr.X, tr.y)
print("decomp", m.n_iter_, m.stop_reason_, flush=True)
c = CascadeSVM(topology="star").fit(tr.X, tr.y, world=2, device="cuda", transport="loopback")
print("cascade", c.result.rounds if hasattr(c.result, "rounds") else "", flush=True)
labels = np.random.default_rng(0).integers(0, 4, size=5000)
o = OneVsRestSVC(device="cuda").fit(tr.X[:5000], labels)
print("ovr", list(o.n_iter_), flush=True)
