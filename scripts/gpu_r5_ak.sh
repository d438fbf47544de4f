#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5ak
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_cases.py -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/r5ak/pytest.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r5ak/pytest.txt | tail -30; exit $rc
