#!/bin/bash
# Row-cache persistent solver: per-phase stamps (SVM355_PSMO_STAMP=1) at 60k / 120k / 250k, over the
# early (miss-heavy) epochs 200.. and a late window (epochs 10000..), then plain timings.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
SVM355_PSMO_STAMP=1 timeout -k 10 300 python -u scripts/rowcache_trace_stats.py 60000 120000 250000 \
  > gpurun_out/rc_stamps.txt 2>&1 &&
SVM355_PSMO_STAMP=1 SVM355_PSMO_STAMP_FROM=10000 timeout -k 10 300 python -u scripts/rowcache_trace_stats.py 60000 120000 250000 \
  > gpurun_out/rc_stamps_late.txt 2>&1 &&
timeout -k 10 300 python -u scripts/rowcache_trace_stats.py 60000 120000 250000 > gpurun_out/rc_plain.txt 2>&1; rc=$?
grep -h "n=\|stamps" gpurun_out/rc_stamps.txt gpurun_out/rc_stamps_late.txt gpurun_out/rc_plain.txt
exit $rc
