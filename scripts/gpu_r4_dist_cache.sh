#!/bin/bash
# Distributed decomposition rehearsals with the column cache forced on (per-rank slices).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_decomp.py -k distributed \
  > gpurun_out/r4dc_pytest.txt 2>&1 || { tail -30 gpurun_out/r4dc_pytest.txt; exit 1; }
tail -8 gpurun_out/r4dc_pytest.txt
