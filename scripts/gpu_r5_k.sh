#!/bin/bash
# Round 5: the per-process decomposition's preflight + gloo fallback, and the bench tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5k
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r5k/pytest.txt 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r5k/pytest.txt | tail -12; exit $rc
