#!/bin/bash
# Round 6: one-vs-rest concurrency at 60k -- every class alone, then all ten at once under a kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6q
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6q/prof -o run -- python3 scripts/ovr_timeline.py > gpurun_out/r6q/ovr.log 2>&1 \
  || { tail -20 gpurun_out/r6q/ovr.log; exit 1; }
grep -E "^class|^sum|^ovr" gpurun_out/r6q/ovr.log
python3 scripts/rocpd_timeline.py gpurun_out/r6q/prof/run_results.db --kernel ws_inner_kernel --window-ms 400 > gpurun_out/r6q/timeline.txt 2>&1
cat gpurun_out/r6q/timeline.txt
