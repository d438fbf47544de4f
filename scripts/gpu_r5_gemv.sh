#!/bin/bash
# Round 5: GEMV time against the number of 64-column halves (kernel trace).
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r5gemv
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/r5gemv/prof -o run -- python3 $R/scripts/gemv_halves_probe.py \
  > $R/gpurun_out/r5gemv/log.txt 2>&1
rc=$?; tail -n 6 $R/gpurun_out/r5gemv/log.txt; exit $rc
