#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 bench_kernels/mfma_f64_peak > gpurun_out/mfma_peak.txt 2>&1; cat gpurun_out/mfma_peak.txt
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_gram.py 60000 > gpurun_out/gram.txt 2>&1; rc=$?
cat gpurun_out/gram.txt
exit $rc
