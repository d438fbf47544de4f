#!/bin/bash
# Round 3 check J: distributed decomposition SMO (rehearsal + process rank) against the one-GPU solve.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decomp.py -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/r3j_decomp_pytest.txt 2>&1; rc=$?
tail -14 gpurun_out/r3j_decomp_pytest.txt
[ $rc -eq 0 ] || { grep -B3 -A40 "Error\|FAILED" gpurun_out/r3j_decomp_pytest.txt | head -80; exit $rc; }
