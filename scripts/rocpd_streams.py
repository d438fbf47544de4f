#!/usr/bin/env python3
"""Per-stream kernel totals from a rocprofv3 results database (rocpd): with P thread ranks rehearsed on
one GPU every rank has its own stream, so this splits a distributed run's device time per rank and per
kernel (replicated kernels cost the same on every rank, divided ones ~1/P).  The ranks' streams are the
P busiest; the per-kernel table shows each kernel's max over those streams (the critical path's share).
Usage: rocpd_streams.py DB [--ranks P] [--top N] [--exclude IDS]"""
import argparse
import collections
import re
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--ranks", type=int, default=0)
ap.add_argument("--top", type=int, default=16)
ap.add_argument("--exclude", default="", help="comma-separated stream ids to leave out (e.g. the one-GPU baseline fit's)")
a = ap.parse_args()
con = sqlite3.connect(a.db)
cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
key = next((c for c in ("stream_id", "queue_id", "stream", "queue") if c in cols), None)
if key is None:
    raise SystemExit(f"no stream column in kernels: {cols}")
rows = list(con.execute(f"select name, start, end, {key} from kernels order by start"))


def short(n):
    n = re.sub(r"^void ", "", n)
    n = n.replace("svm355::(anonymous namespace)::", "").replace("svm355::", "")
    m = re.match(r"([A-Za-z_0-9]+(<[^()]*>)?)", n)
    return (m.group(1) if m else n)[:70]


per = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0]))
for n, s, e, st in rows:
    v = per[st][short(n)]
    v[0] += 1
    v[1] += (e - s) / 1e6
busy = {st: sum(v[1] for v in d.values()) for st, d in per.items()}
ex = {int(x) for x in a.exclude.split(",") if x}
streams = sorted((s for s in busy if s not in ex), key=lambda s: -busy[s])
if a.ranks:
    streams = streams[: a.ranks]
print(f"{key}: " + "  ".join(f"{s}={busy[s]:.1f} ms" for s in streams))
names = collections.Counter()
for s in streams:
    for k, v in per[s].items():
        names[k] = max(names[k], v[1])
print(f"{'kernel':70s} {'max ms':>9s} {'min ms':>9s} {'calls/rank':>10s}")
for k, mx in names.most_common(a.top):
    mn = min(per[s][k][1] if k in per[s] else 0.0 for s in streams)
    calls = max(per[s][k][0] if k in per[s] else 0 for s in streams)
    print(f"{k:70s} {mx:9.2f} {mn:9.2f} {calls:10d}")
