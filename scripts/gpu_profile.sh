#!/bin/bash
# Kernel-level profile (rocprofv3 --kernel-trace --stats) of the 1-GPU bench + a wall-clock breakdown of SVC.fit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/fit_breakdown.py > gpurun_out/fit_breakdown.txt 2>&1 || { cat gpurun_out/fit_breakdown.txt; exit 1; }
cat gpurun_out/fit_breakdown.txt
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_stdout.txt 2>&1 || { tail -20 gpurun_out/prof_stdout.txt; exit 1; }
tail -2 gpurun_out/prof_stdout.txt
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats.csv
cut -c1-220 gpurun_out/kernel_stats.csv | head -20
