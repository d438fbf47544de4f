#!/bin/bash
# Sort-free working-set build: oracle / decomposition / distributed tests, then fit timings and kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_decomp_oracle.py \
  tests/test_gpu_decomp.py > gpurun_out/r4b_pytest.txt 2>&1 || { tail -30 gpurun_out/r4b_pytest.txt; exit 1; }
tail -3 gpurun_out/r4b_pytest.txt
timeout -k 10 400 python -u scripts/decomp_cache_timing.py 60000 250000 1000000 > gpurun_out/r4cache_time.txt 2>&1 \
  || { tail -20 gpurun_out/r4cache_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4cache_time.txt
CACHES=1 bash scripts/gpu_r4_cache_prof.sh 1000000 || exit 1
CACHES=1 bash scripts/gpu_r4_cache_prof.sh 250000 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4wwprof -o run -- \
  python3 bench.py --steps 10 --warmup 3 --decomp-fits 0 --f64-fits 0 > gpurun_out/r4wwprof.log 2>&1 || { tail -5 gpurun_out/r4wwprof.log; exit 1; }
