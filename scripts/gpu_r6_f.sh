#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/newton_probe.py > gpurun_out/r6f_probe.txt 2>&1 || { cat gpurun_out/r6f_probe.txt; exit 1; }
cat gpurun_out/r6f_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp_oracle.py tests/test_gpu_decomp.py -x -v --timeout 300 --timeout-method thread \
  -k "newton or device_trajectory or real_valued or rehearsal_equals" > gpurun_out/r6f_pytest.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r6f_pytest.txt; exit 1; }
tail -2 gpurun_out/r6f_pytest.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread \
  -k "real_valued or refuses or allowed" > gpurun_out/r6f_pytest_bench.txt 2>&1 || { echo "bench pytest failed"; tail -60 gpurun_out/r6f_pytest_bench.txt; exit 1; }
tail -2 gpurun_out/r6f_pytest_bench.txt
timeout -k 10 500 python -u scripts/shrink_sweep.py 60000 '' 'SVM355_DECOMP_NEWTON=0' 'SVM355_DECOMP_NEWTON_EVERY=100' \
  'SVM355_DECOMP_NEWTON_EVERY=100 SVM355_DECOMP_NEWTON_REPEAT=1' 'SVM355_DECOMP_NEWTON_REPEAT=1' > gpurun_out/r6f_sweep.txt 2>&1
cat gpurun_out/r6f_sweep.txt
