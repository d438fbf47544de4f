#!/bin/bash
# Round 6: one-vs-rest concurrency at 60k with more hardware queues per process (GPU_MAX_HW_QUEUES,
# HIP's default 4): ten class streams on 4 in-order queues run at most 4 kernels at once.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6r
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for q in 4 10 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6r/prof_q$q -o run -- python3 scripts/ovr_timeline.py > gpurun_out/r6r/ovr_q$q.log 2>&1 \
    || { tail -20 gpurun_out/r6r/ovr_q$q.log; exit 1; }
  echo "== GPU_MAX_HW_QUEUES=$q"; grep -E "^sum|^ovr" gpurun_out/r6r/ovr_q$q.log
  python3 scripts/rocpd_timeline.py gpurun_out/r6r/prof_q$q/run_results.db --kernel ws_inner_kernel --window-ms 150 | head -2
done
for q in 4 10 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 scripts/ovr_workers_probe.py > gpurun_out/r6r/workers_q$q.txt 2>&1 || { tail -20 gpurun_out/r6r/workers_q$q.txt; exit 1; }
  echo "== workers, GPU_MAX_HW_QUEUES=$q"; grep workers gpurun_out/r6r/workers_q$q.txt
done
