#!/bin/bash
# Round 5: PMC counters of the decomposition kernels in the bench (GEMV, inner solve, column store),
# two passes of at most 8 SQ counters each, counters only (no trace domains).
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r5pmc
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU \
  --kernel-include-regex "igram_tri_kernel|ws_inner_kernel|igram_colstore_narrow" -f csv -d $R/gpurun_out/r5pmc/p1 -o run \
  -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/r5pmc/p1.log 2>&1
rc=$?; echo "pass1 rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM \
  --kernel-include-regex "igram_tri_kernel|ws_inner_kernel|igram_colstore_narrow" -f csv -d $R/gpurun_out/r5pmc/p2 -o run \
  -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/r5pmc/p2.log 2>&1
rc=$?; echo "pass2 rc $rc"; find $R/gpurun_out/r5pmc -name "*.csv" | head; exit $rc
