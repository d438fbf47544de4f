#!/bin/bash
# Row-cache persistent solver profile: GPU tests, plain timings 60k..1M (distinct rows, misses), and
# per-phase stamps over the miss-heavy early window (epochs 200..) and a hits-only window (10000..).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "row_cache" \
  > gpurun_out/rcp_pytest.txt 2>&1 || { tail -30 gpurun_out/rcp_pytest.txt; exit 1; }
tail -1 gpurun_out/rcp_pytest.txt
timeout -k 10 400 python -u scripts/rowcache_trace_stats.py 60000 120000 250000 500000 1000000 > gpurun_out/rcp_plain.txt 2>&1 || exit 1
SVM355_PSMO_STAMP=1 timeout -k 10 300 python -u scripts/rowcache_trace_stats.py 60000 250000 > gpurun_out/rcp_stamps.txt 2>&1 || exit 1
SVM355_PSMO_STAMP=1 SVM355_PSMO_STAMP_FROM=10000 timeout -k 10 300 python -u scripts/rowcache_trace_stats.py 60000 250000 \
  > gpurun_out/rcp_stamps_late.txt 2>&1 || exit 1
grep -h "n=\|stamps" gpurun_out/rcp_plain.txt gpurun_out/rcp_stamps.txt gpurun_out/rcp_stamps_late.txt
