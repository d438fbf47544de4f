#!/bin/bash
# rocprofv3 kernel trace + stats of the native single-GPU trainer (60k synthetic MNIST).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${1:-60000}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  svm355/bin/svm_gpu --synthetic $N,10000 --quiet > gpurun_out/prof_stdout.txt 2>&1 || { tail -20 gpurun_out/prof_stdout.txt; exit 1; }
cat gpurun_out/prof_stdout.txt | tail -12
find gpurun_out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats.csv
head -20 gpurun_out/kernel_stats.csv
