#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/newton_probe.py > gpurun_out/r6g_probe.txt 2>&1 || { cat gpurun_out/r6g_probe.txt; exit 1; }
cat gpurun_out/r6g_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp_oracle.py -x -v --timeout 300 --timeout-method thread \
  -k "newton" > gpurun_out/r6g_pytest.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r6g_pytest.txt; exit 1; }
tail -2 gpurun_out/r6g_pytest.txt
timeout -k 10 500 python -u scripts/shrink_sweep.py 60000 '' 'SVM355_DECOMP_NEWTON=0' 'SVM355_DECOMP_NEWTON_EVERY=100' \
  'SVM355_DECOMP_NEWTON_EVERY=100 SVM355_DECOMP_NEWTON_REPEAT=1' 'SVM355_DECOMP_NEWTON_FRAC=9' > gpurun_out/r6g_sweep.txt 2>&1
cat gpurun_out/r6g_sweep.txt
