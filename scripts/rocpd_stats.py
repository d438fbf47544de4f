#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 SQLite results database (rocpd), for the dispatches from the
`skip`-th occurrence of a marker kernel on (e.g. the second fit: --marker ws_init_kernel --skip 1).
Usage: rocpd_stats.py DB [--marker NAME --skip K] [--top N]"""
import argparse
import collections
import re
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--marker", default=None)
ap.add_argument("--skip", type=int, default=0)
ap.add_argument("--until", default=None, help="stop at the next occurrence of this kernel after the start")
ap.add_argument("--top", type=int, default=25)
a = ap.parse_args()
con = sqlite3.connect(a.db)
rows = list(con.execute("select name, start, end from kernels order by start"))


def short(n):
    n = re.sub(r"^void ", "", n)
    n = n.replace("svm355::(anonymous namespace)::", "").replace("svm355::", "")
    m = re.match(r"([A-Za-z_0-9]+(<[^()]*>)?)", n)
    return (m.group(1) if m else n)[:90]


start = 0
if a.marker:
    hits = [i for i, r in enumerate(rows) if short(r[0]).startswith(a.marker)]
    start = hits[a.skip]
seg = rows[start:]
if a.until:
    for j in range(1, len(seg)):
        if short(seg[j][0]).startswith(a.until):
            seg = seg[:j]
            break
tot = collections.defaultdict(lambda: [0, 0.0])
for n, s, e in seg:
    k = short(n)
    tot[k][0] += 1
    tot[k][1] += (e - s) / 1e6
span = (seg[-1][2] - seg[0][1]) / 1e6
busy = sum(v[1] for v in tot.values())
print(f"dispatches {len(seg)}  span {span:.3f} ms  busy {busy:.3f} ms")
for k, v in sorted(tot.items(), key=lambda x: -x[1][1])[: a.top]:
    print(f"{v[1]:10.3f} ms {v[0]:6d} {1e3 * v[1] / v[0]:9.1f} us  {k}")
