#!/bin/bash
# Persistent row-cache solver: its GPU tests, then the large-n timings (rows touched, misses).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -k "row_cache" \
  > gpurun_out/pytest_rc.txt 2>&1; rc=$?
tail -12 gpurun_out/pytest_rc.txt
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/pytest_rc.txt | head -60; exit $rc; }
timeout -k 10 300 python -u scripts/rowcache_trace_stats.py 60000 120000 250000 2>&1 | grep "n=" | tee gpurun_out/rowcache_persistent.txt
