#!/bin/bash
# Round 4: the explicitly loaded RCCL (rccl_api.h) under every RCCL test, the per-solve cascade solver.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_cascade.py tests/test_gpu_bench.py tests/test_gpu_decomp.py \
  tests/test_gpu_dsmo.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4c_pytest.txt 2>&1 \
  || { tail -60 gpurun_out/r4c_pytest.txt; exit 1; }
tail -3 gpurun_out/r4c_pytest.txt
grep -h "rccl" gpurun_out/r4c_pytest.txt | head -5
