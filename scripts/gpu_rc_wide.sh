#!/bin/bash
# Row-cache persistent solver with wider teams (2 / 4 records per sweep lane): tests, then timings at
# 250k for team caps 64 / 128 / 256, and n = 500k / 1M (beyond the 64-workgroup shapes).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -k "row_cache" \
  > gpurun_out/pytest_rc_wide.txt 2>&1; rc=$?
tail -4 gpurun_out/pytest_rc_wide.txt
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/pytest_rc_wide.txt | head -60; exit $rc; }
for m in 64 128 256; do
  SVM355_RC_MAXG=$m timeout -k 10 200 python -u scripts/rowcache_trace_stats.py 250000 2>&1 | grep "n=" | sed "s/^/maxg=$m /" || exit 1
done | tee gpurun_out/rc_wide_250k.txt
timeout -k 10 400 python -u scripts/rowcache_trace_stats.py 500000 1000000 2>&1 | grep "n=" | tee gpurun_out/rc_wide_large.txt
