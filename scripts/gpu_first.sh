#!/bin/bash
# First GPU contact: CLI parity vs serial on small synthetic data, then a 60k run.
set -o pipefail
cd "$(dirname "$0")/.."
B=svm355/bin
mkdir -p gpurun_out
timeout -k 10 120 $B/svm_gpu --synthetic 3000,1000 > gpurun_out/gpu_3k.txt 2>&1 || { echo "3k failed: $?"; cat gpurun_out/gpu_3k.txt; exit 1; }
cat gpurun_out/gpu_3k.txt
timeout -k 10 300 $B/svm_gpu --synthetic 20000,10000 > gpurun_out/gpu_20k.txt 2>&1 || { echo "20k failed: $?"; cat gpurun_out/gpu_20k.txt; exit 1; }
cat gpurun_out/gpu_20k.txt
timeout -k 10 400 $B/svm_gpu --synthetic 60000,10000 --json gpurun_out/gpu_60k.json > gpurun_out/gpu_60k.txt 2>&1 || { echo "60k failed: $?"; cat gpurun_out/gpu_60k.txt; exit 1; }
cat gpurun_out/gpu_60k.txt
