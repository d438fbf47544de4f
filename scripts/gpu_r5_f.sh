#!/bin/bash
# Round 5: the cold upload's steps with and without the staging ring, the GPU suites touched this round,
# and the 1M cascade rehearsal (star P = 8, every solve timed alone) against today's 1-GPU default.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5f
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/upload_probe.py > gpurun_out/r5f/upload_staged.txt 2>&1 &&
SVM355_H2D_STAGING=0 timeout -k 10 120 python3 scripts/upload_probe.py > gpurun_out/r5f/upload_direct.txt 2>&1 &&
grep -E "^[0-9] " gpurun_out/r5f/upload_staged.txt gpurun_out/r5f/upload_direct.txt &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_decomp.py tests/test_gpu_cascade.py tests/test_gpu_cli.py \
  tests/test_gpu_dsmo.py tests/test_gpu_decomp_oracle.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5f/pytest.txt 2>&1 &&
tail -2 gpurun_out/r5f/pytest.txt &&
SVM355_CASCADE_RELEASE_GRAM=1 timeout -k 10 700 python -u -m svm355 scale --trainer cascade --transport loopback \
  --ranks 8 --sizes 1000000 --test-rows 2000 --repeats 1 --warmup 0 --json gpurun_out/r5f/cascade_1m.json \
  > gpurun_out/r5f/cascade_1m.txt 2>&1; rc=$?; tail -8 gpurun_out/r5f/cascade_1m.txt; exit $rc
