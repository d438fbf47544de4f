#!/bin/bash
# Round 5: the distributed decomposition's P-GPU critical path at 3M rows (loopback ranks on one GPU,
# every rank's device work timed alone), with the streamed selection and the evicting column cache.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5as
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5as/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r5as/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m svm355 scale --transport loopback --ranks 1,2,4,8 --sizes 3000000 \
  --max-iter 10000000 --test-rows 2000 --repeats 1 --warmup 1 --json gpurun_out/r5as/scale_3m.json \
  > gpurun_out/r5as/scale.txt 2>&1
rc=$?; tail -12 gpurun_out/r5as/scale.txt; exit $rc
