#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_cascade.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_cascade.txt 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu_cascade.txt
[ $rc -eq 0 ] || { grep -B5 -A30 "FAIL\|Error" gpurun_out/pytest_gpu_cascade.txt | head -80; exit $rc; }
timeout -k 10 250 python -u scripts/cascade_overhead.py 1 > gpurun_out/cascade_overhead.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/cascade_overhead.txt | tail -4
