#!/bin/bash
# Round 6: kernel census of the final 1-GPU bench (defaults), for profiles/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6m
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6m/prof -o run -- python3 bench.py --steps 5 --warmup 1 \
  --baseline-1gpu 0 --out gpurun_out/r6m/bench.json > gpurun_out/r6m/prof.log 2>&1 || { tail -20 gpurun_out/r6m/prof.log; exit 1; }
python3 scripts/rocpd_stats.py gpurun_out/r6m/prof/run_results.db --marker ws_init_kernel --skip 2 --until ws_init_kernel --top 20 > gpurun_out/r6m/stats_fit.txt 2>&1
cat gpurun_out/r6m/stats_fit.txt
