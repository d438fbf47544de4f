#!/bin/bash
# PMC passes (one counter group per run) over the exact-integer Gram kernel.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/pmc_gram
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum" \
           "TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_64B_sum" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_WAIT_ANY SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_gram/p$i -o p$i -- python3 $R/scripts/gram_once.py > $R/gpurun_out/pmc_gram/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_gram/p$i.log; exit 1; }
  echo "pass $i ok"
done
