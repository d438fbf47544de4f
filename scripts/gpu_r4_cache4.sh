#!/bin/bash
# Round 4: column cache (grouped reader, streamed narrow store): oracle / identity tests, timings,
# kernel stats at 1M.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_decomp_oracle.py \
  > gpurun_out/r4cache_pytest.txt 2>&1 || { tail -30 gpurun_out/r4cache_pytest.txt; exit 1; }
timeout -k 10 400 python -u scripts/decomp_cache_timing.py 60000 250000 1000000 > gpurun_out/r4cache_time.txt 2>&1 \
  || { tail -20 gpurun_out/r4cache_time.txt; exit 1; }
CACHES=1 bash scripts/gpu_r4_cache_prof.sh 1000000 || exit 1
CACHES=1 bash scripts/gpu_r4_cache_prof.sh 250000 || exit 1
[ -n "$PMC" ] && { bash scripts/gpu_r4_narrow_pmc.sh || exit 1; }
grep -v amdgpu.ids gpurun_out/r4cache_time.txt
tail -3 gpurun_out/r4cache_pytest.txt
