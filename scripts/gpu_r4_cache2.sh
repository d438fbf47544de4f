#!/bin/bash
# Round 4: column cache v2 (narrow store at 4 waves/SIMD) -- tests, timings, profiles, working-set sweep.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_decomp_oracle.py \
  > gpurun_out/r4cache_pytest.txt 2>&1 || { tail -30 gpurun_out/r4cache_pytest.txt; exit 1; }
timeout -k 10 400 python -u scripts/decomp_cache_timing.py 250000 1000000 > gpurun_out/r4cache_time.txt 2>&1 \
  || { tail -20 gpurun_out/r4cache_time.txt; exit 1; }
CACHES=1 bash scripts/gpu_r4_cache_prof.sh 1000000 || exit 1
for n in 250000 1000000; do for q in 384 512 640 768; do
  timeout -k 10 120 python -u scripts/decomp_inner_probe.py $n $q >> gpurun_out/r4cache_qsweep.txt 2>&1 || exit 1
done; done
cat gpurun_out/r4cache_time.txt gpurun_out/r4cache_qsweep.txt
tail -3 gpurun_out/r4cache_pytest.txt
