#!/bin/bash
# Round 3: decomposition GPU tests (incl. the rejected inner stop fraction).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/dtests2.txt 2>&1 || { tail -40 gpurun_out/dtests2.txt; exit 1; }
tail -15 gpurun_out/dtests2.txt
