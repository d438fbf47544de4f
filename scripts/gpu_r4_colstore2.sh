#!/bin/bash
# Column store (operand-swapped narrow kernel): unit tests, per-m timing, fit timings.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_decomp_oracle.py \
  > gpurun_out/r4cs_pytest.txt 2>&1 || { tail -30 gpurun_out/r4cs_pytest.txt; exit 1; }
for m in 1 8 16 32 64; do
  SVM355_GEMV_VIA_CACHE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4cs_$m -o run \
    -- python3 scripts/colstore_bench.py 1000000 $m > gpurun_out/r4cs_$m.log 2>&1 || { tail -5 gpurun_out/r4cs_$m.log; exit 1; }
done
timeout -k 10 400 python -u scripts/decomp_cache_timing.py 60000 250000 1000000 > gpurun_out/r4cache_time.txt 2>&1 \
  || { tail -20 gpurun_out/r4cache_time.txt; exit 1; }
CACHES=1 bash scripts/gpu_r4_cache_prof.sh 1000000 || exit 1
CACHES=1 bash scripts/gpu_r4_cache_prof.sh 250000 || exit 1
grep -v amdgpu.ids gpurun_out/r4cache_time.txt
tail -3 gpurun_out/r4cs_pytest.txt
