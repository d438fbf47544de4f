#!/bin/bash
# Round 5: extra-group flushes fused into one FMA at every K site -- numerics and bit-agreement
# tests (kernels, decomposition + oracles, pairwise), then the 1-GPU bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5l
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_decomp_oracle.py tests/test_gpu_decomp.py \
  tests/test_gpu_dsmo.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5l/pytest.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r5l/pytest.txt | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5l/bench.json 2> gpurun_out/r5l/bench.err
rc=$?; tail -c 1500 gpurun_out/r5l/bench.json; exit $rc
