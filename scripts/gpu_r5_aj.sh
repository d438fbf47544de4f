#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5aj
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r5aj/pytest.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r5aj/pytest.txt | tail -12; exit $rc
