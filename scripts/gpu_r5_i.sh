#!/bin/bash
# Round 5: the bench's N > 1 line survives a failing post-headline cascade; the per-process tests again
# (HostCommRank now on its own gloo group).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5i
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r5i/pytest.txt 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r5i/pytest.txt | tail -12; exit $rc
