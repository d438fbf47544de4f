#!/bin/bash
# Second pair's j by the second-order gain of row i2 (SVM355_DECOMP_WSS=4) against the first-order j2 (3):
# oracle tests, then fit times.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_decomp_oracle.py \
  > gpurun_out/r4j2s_pytest.txt 2>&1 || { tail -30 gpurun_out/r4j2s_pytest.txt; exit 1; }
tail -2 gpurun_out/r4j2s_pytest.txt
SVM355_TIMING_VAR=SVM355_DECOMP_WSS SVM355_TIMING_VALUES=3,4,3,4 \
  timeout -k 10 500 python -u scripts/decomp_cache_timing.py ${SIZES:-40000 60000 120000 250000 1000000} 2>&1 | grep -v amdgpu.ids | grep "cache="
