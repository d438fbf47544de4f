#!/bin/bash
# Round 5: one-vs-rest defaults to the decomposition solver per class -- OvR GPU tests, the CLI, the probe.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5t
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "ovr" -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5t/pytest.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r5t/pytest.txt | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m svm355 multiclass --synthetic 60000,10000 --json gpurun_out/r5t/mc.json > gpurun_out/r5t/mc.txt 2>&1
rc=$?; cat gpurun_out/r5t/mc.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ovr_decomp_probe.py 60000 > gpurun_out/r5t/ovr.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5t/ovr.txt | tail -12; exit $rc
