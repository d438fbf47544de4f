#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5ai
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -k "not_dividing" -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5ai/pytest.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r5ai/pytest.txt | tail -5; exit $rc
