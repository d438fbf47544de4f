#!/usr/bin/env python3
"""Per-solve log of a cascade rehearsal on one GPU (thread ranks over loopback, each solve timed alone):
rank, round, layer, rows, pair updates, decomposition outer iterations, solo ms.

    SVM355_CASCADE_SERIAL_SOLVES=1 python scripts/cascade_solve_log.py 60000 star 2 decomp
"""
import os
import sys

from svm355 import SVMParams
from svm355.parallel.cascade import CascadeSVM, critical_path
from svm355.parallel.rccl import DeviceGroup
from svm355.utils.data import synthetic_mnist

n, topo, P, solver = int(sys.argv[1]), sys.argv[2], int(sys.argv[3]), sys.argv[4]
tr = synthetic_mnist(n, seed=2024).compact()
g = DeviceGroup(P, "loopback")
c = CascadeSVM(SVMParams(), topology=topo, solver=solver)
c.fit(tr.X, tr.y, world=P, device="cuda", group=g)  # warm
c.fit(tr.X, tr.y, world=P, device="cuda", group=g)
r = c.result
print(f"{solver} {topo} P={P}: rounds {r.rounds} n_sv {len(r.ids)} critical path {critical_path(r.solves, topo)[1]} ms")
for s in sorted(r.solves, key=lambda s: (s["round"], s["layer"] != "local", s["rank"])):
    print(f"  r{s['round']} {s['layer']:>7} rank {s['rank']} n {s['n']:6d} it {s['iterations']:6d} outer {s['outer']:4d} "
          f"solo {s['solo_ms']:8.3f} ms skipped {int(s['skipped'])}")
g.close()
