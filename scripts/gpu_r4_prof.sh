#!/bin/bash
# rocprofv3 kernel trace + stats of the 1-GPU headline bench (decomposition solver, 60k).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4prof -o run \
  -- python3 bench.py --steps 5 --warmup 2 --decomp-fits 0 --f64-fits 0 > gpurun_out/r4prof.log 2>&1 \
  || { tail -20 gpurun_out/r4prof.log; exit 1; }
f=$(find gpurun_out/r4prof -name "*kernel_stats.csv" | head -1); echo "stats: $f"; head -14 "$f" | cut -c1-200
t=$(find gpurun_out/r4prof -name "*kernel_trace.csv" | head -1); echo "trace: $t"; ls -la "$t"
