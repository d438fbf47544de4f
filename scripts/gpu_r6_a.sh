#!/bin/bash
# Round 6: shrinking -- device vs oracle GPU tests, then fit times with and without shrinking.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp_oracle.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r6a_pytest.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r6a_pytest.txt; exit 1; }
tail -5 gpurun_out/r6a_pytest.txt
timeout -k 10 400 python -u scripts/shrink_sweep.py 60000,250000 '' 'SVM355_DECOMP_SHRINK=0' \
  'SVM355_DECOMP_SHRINK=1' 'SVM355_DECOMP_SHRINK_MARGIN=1' > gpurun_out/r6a_sweep.txt 2>&1
cat gpurun_out/r6a_sweep.txt
timeout -k 10 300 python -u scripts/shrink_sweep.py 1000000 '' 'SVM355_DECOMP_SHRINK=0' > gpurun_out/r6a_sweep_1m.txt 2>&1
cat gpurun_out/r6a_sweep_1m.txt
