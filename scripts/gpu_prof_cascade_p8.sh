#!/bin/bash
# rocprofv3 kernel stats of the 8-rank star cascade rehearsal (loopback, one GPU): which kernels the
# cascade's local solves and rank-0 merges run (persistent / single-workgroup SMO, exact-integer Gram,
# KKT skip check, pack / assemble).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
SVM355_CASCADE_SERIAL_SOLVES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_p8 -o run \
  -- python3 bench.py --gpus 8 --transport loopback --steps 1 --warmup 1 --baseline-1gpu 0 > gpurun_out/prof_p8.log 2>&1 \
  || { tail -20 gpurun_out/prof_p8.log; exit 1; }
f=$(find gpurun_out/prof_p8 -name "*kernel_stats.csv" | head -1); echo "stats: $f"; head -16 "$f" | cut -c1-160
