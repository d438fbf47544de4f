#!/bin/bash
# Round 5: one-vs-rest decomposition with more hardware queues than HIP's default 4 (10 class streams).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5ac
export TMPDIR=/tmp
for q in 4 8 12; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u scripts/ovr_workers_probe.py > gpurun_out/r5ac/q$q.txt 2>&1 || exit $?
  echo "GPU_MAX_HW_QUEUES=$q"; grep workers gpurun_out/r5ac/q$q.txt
done
