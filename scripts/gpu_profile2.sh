#!/bin/bash
# rocprofv3 kernel trace + roctx marker ranges of the 1-GPU bench; then the GPU test suite.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof2
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof2_stdout.txt 2>&1 || { tail -20 gpurun_out/prof2_stdout.txt; exit 1; }
grep metric gpurun_out/prof2_stdout.txt | cut -c1-200
find gpurun_out/prof2 -name "*.csv" | head -20
f=$(find gpurun_out/prof2 -name "*kernel_stats.csv" | head -1); cut -c1-200 "$f" | head -12
m=$(find gpurun_out/prof2 -name "*marker_api_trace.csv" | head -1); [ -n "$m" ] && head -3 "$m" && wc -l "$m"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.txt; exit $rc
