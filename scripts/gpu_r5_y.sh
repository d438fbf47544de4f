#!/bin/bash
# Round 5: one-vs-rest GPU tests after the pool threads hand their slabs back; the OvR probe.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5y
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "ovr" -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5y/pytest.txt 2>&1
rc=$?; tail -n 2 gpurun_out/r5y/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ovr_decomp_probe.py 60000 > gpurun_out/r5y/ovr.txt 2>&1
rc=$?; grep -E "fit|agreement" gpurun_out/r5y/ovr.txt; exit $rc
