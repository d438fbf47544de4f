#!/bin/bash
# Round 5: candidate rows loaded before the folds (ws_inner_kernel SPEC) -- oracle bit-identity, then
# fit time with and without (SVM355_DECOMP_SPEC=0) at 60k / 250k, and the phase ticks.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5q
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp_oracle.py tests/test_gpu_decomp.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r5q/pytest.txt 2>&1
rc=$?; tail -n 3 gpurun_out/r5q/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/decomp_env_sweep.py 60000,250000 '' 'SVM355_DECOMP_SPEC=0' '' 'SVM355_DECOMP_SPEC=0' \
  > gpurun_out/r5q/sweep.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5q/sweep.txt; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=. SVM355_DECOMP_PROF=1 timeout -k 10 200 python -u scripts/decomp_inner_probe.py 60000 1024 > gpurun_out/r5q/prof.txt 2>&1
rc=$?; tail -n 3 gpurun_out/r5q/prof.txt; exit $rc
