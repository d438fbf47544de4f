#!/bin/bash
# Round 5: L2 traffic of the decomposition kernels (is the f-update GEMV memory-bound?): one pass with
# TCC_HIT/MISS/EA0_RDREQ (3 TCC), TCP_TCC_READ_REQ (TCP), TA busy (TA), counters only.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r5pmc2
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr \
  --kernel-include-regex "igram_tri_kernel|ws_inner_kernel|igram_colstore_narrow" -f csv -d $R/gpurun_out/r5pmc2/p -o run \
  -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/r5pmc2/p.log 2>&1
rc=$?; echo "rc $rc"; tail -n 3 $R/gpurun_out/r5pmc2/p.log; exit $rc
