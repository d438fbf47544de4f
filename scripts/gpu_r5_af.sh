#!/bin/bash
# Round 5: one-vs-rest save / load on the GPU.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5af
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "ovr" -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5af/pytest.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r5af/pytest.txt | tail -14; exit $rc
