#!/usr/bin/env python3
"""Summarise a rocprofv3 marker trace (csv): each svm355.* range with its duration and the kernel
time inside it.    python scripts/trace_summary.py <dir with run_marker_api_trace.csv>"""
import csv
import glob
import sys

d = sys.argv[1]
mk = glob.glob(f"{d}/**/*marker_api_trace.csv", recursive=True)
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(mk[0]))) if mk else []
kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(kt[0]))] if kt else []
for r in rows:
    name = r.get("Function") or r.get("Operation") or ""
    msg = r.get("Message") or r.get("Name") or name
    if "svm355" not in msg:
        continue
    t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy = sum(min(e, t1) - max(s, t0) for s, e in kern if e > t0 and s < t1)
    print(f"{msg:55s} {(t1 - t0) / 1e6:9.2f} ms  kernels {busy / 1e6:9.2f} ms")
if not rows:
    print("no marker rows; files:", glob.glob(f"{d}/**/*.csv", recursive=True))
