#!/usr/bin/env python3
"""HIP runtime API calls from a rocprofv3 --runtime-trace results database (rocpd): totals per call name,
and the slowest single calls in time order with their offset from the first call.
Usage: rocpd_api.py DB [--top N] [--min-ms X]"""
import argparse
import collections
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--top", type=int, default=20)
ap.add_argument("--min-ms", type=float, default=2.0)
a = ap.parse_args()
con = sqlite3.connect(a.db)
names = [r[0] for r in con.execute("select name from sqlite_master where type in ('table', 'view')")]
view = next((v for v in ("regions", "region") if v in names), None)
if view is None:
    print("no region view; tables/views:", names)
    raise SystemExit(0)
cols = [r[1] for r in con.execute(f"pragma table_info({view})")]
cat = "category" if "category" in cols else None
q = f"select name, start, end{', ' + cat if cat else ''} from {view} order by start"
rows = list(con.execute(q))
if not rows:
    raise SystemExit("no API records")
t0 = rows[0][1]
tot = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    tot[r[0]][0] += 1
    tot[r[0]][1] += (r[2] - r[1]) / 1e6
print(f"{len(rows)} API records over {(rows[-1][2] - t0) / 1e6:.1f} ms")
for k, v in sorted(tot.items(), key=lambda x: -x[1][1])[: a.top]:
    print(f"{v[1]:10.3f} ms {v[0]:7d}  {k}")
print(f"single calls above {a.min_ms} ms (offset from the first record):")
for r in rows:
    d = (r[2] - r[1]) / 1e6
    if d >= a.min_ms:
        print(f"  +{(r[1] - t0) / 1e6:9.1f} ms  {d:9.3f} ms  {r[0]}" + (f"  [{r[3]}]" if cat else ""))
