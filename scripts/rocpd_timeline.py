#!/usr/bin/env python3
"""Concurrency of one kernel over the last window of a rocpd kernel trace: from the last occurrence of
--window-start (e.g. the last fit's first kernel) to the end, how long k instances of --kernel ran at once
(k = 0, 1, 2, ...), and each other kernel's busy time in that window.
Usage: rocpd_timeline.py DB --kernel ws_inner_kernel [--window-ms X]"""
import argparse
import collections
import re
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--kernel", default="ws_inner_kernel")
ap.add_argument("--window-ms", type=float, default=0.0, help="only the last X ms of the trace (0: all)")
a = ap.parse_args()
con = sqlite3.connect(a.db)
rows = list(con.execute("select name, start, end from kernels order by start"))
end = max(r[2] for r in rows)
t0 = end - a.window_ms * 1e6 if a.window_ms > 0 else min(r[1] for r in rows)
rows = [r for r in rows if r[2] > t0]


def short(n):
    n = re.sub(r"^void ", "", n).replace("svm355::(anonymous namespace)::", "").replace("svm355::", "")
    m = re.match(r"([A-Za-z_0-9]+)", n)
    return m.group(1) if m else n[:40]


ev = []
busy = collections.defaultdict(float)
for n, s, e in rows:
    s = max(s, t0)
    busy[short(n)] += (e - s) / 1e6
    if short(n).startswith(a.kernel):
        ev += [(s, 1), (e, -1)]
ev.sort()
hist = collections.defaultdict(float)
cur, last = 0, t0
for t, d in ev:
    hist[cur] += (t - last) / 1e6
    cur += d
    last = t
hist[cur] += (end - last) / 1e6
print(f"window {(end - t0) / 1e6:.2f} ms")
print(f"{a.kernel} instances running at once: " + ", ".join(f"{k}: {v:.2f} ms" for k, v in sorted(hist.items())))
for k, v in sorted(busy.items(), key=lambda x: -x[1])[:10]:
    print(f"  {v:9.2f} ms busy  {k}")
