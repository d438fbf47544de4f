#!/bin/bash
# rocprofv3 kernel trace + roctx marker ranges of the 1-GPU bench, the native svm_gpu CLI at 60k, then the GPU suite.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof3
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof3_stdout.txt 2>&1 || { tail -20 gpurun_out/prof3_stdout.txt; exit 1; }
grep metric gpurun_out/prof3_stdout.txt | cut -c1-200
f=$(find gpurun_out/prof3 -name "*kernel_stats.csv" | head -1); cut -c1-200 "$f" | head -14
timeout -k 10 300 ./svm355/bin/svm_gpu --synthetic 60000,10000 --warmup 1 > gpurun_out/svm_gpu_60k.txt 2>&1 || { cat gpurun_out/svm_gpu_60k.txt; exit 1; }
cat gpurun_out/svm_gpu_60k.txt
timeout -k 10 300 ./svm355/bin/svm_cascade --synthetic 60000,10000 --gpus 1 --topology star > gpurun_out/svm_cascade_1.txt 2>&1 || { cat gpurun_out/svm_cascade_1.txt; exit 1; }
tail -8 gpurun_out/svm_cascade_1.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.txt; exit $rc
