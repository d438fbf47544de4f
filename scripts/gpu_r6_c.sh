#!/bin/bash
# Round 6: the Newton polish -- device vs oracle, then fit times.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp_oracle.py -x -v --timeout 300 --timeout-method thread \
  -k "newton or shrinking or device_trajectory or warm_start or column_cache or kww or streamed" > gpurun_out/r6c_pytest.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r6c_pytest.txt; exit 1; }
tail -3 gpurun_out/r6c_pytest.txt
timeout -k 10 500 python -u scripts/shrink_sweep.py 60000 '' 'SVM355_DECOMP_NEWTON=0' 'SVM355_DECOMP_NEWTON=0 SVM355_DECOMP_SHRINK=0' \
  'SVM355_DECOMP_SHRINK=0' 'SVM355_DECOMP_NEWTON_EVERY=25' 'SVM355_DECOMP_NEWTON_EVERY=100' 'SVM355_DECOMP_NEWTON_REPEAT=1' \
  'SVM355_DECOMP_NEWTON_REPEAT=4' > gpurun_out/r6c_sweep.txt 2>&1
cat gpurun_out/r6c_sweep.txt
