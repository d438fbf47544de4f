#!/bin/bash
# python -m svm355 scale on one MI355X: P = 1 on RCCL (2/4/8 skipped: one GPU), then the loopback
# rehearsal of P = 1, 2, 4, 8 (solo device time per solve -> critical path); then rocprofv3 PMC passes
# over the 60k fit (SMO + Gram kernels), one pass per counter group.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m svm355 scale --ranks 1,2 --repeats 3 --json gpurun_out/scale_rccl.json \
  > gpurun_out/scale_rccl.txt 2>&1 || { tail -20 gpurun_out/scale_rccl.txt; exit 1; }
cat gpurun_out/scale_rccl.txt
timeout -k 10 400 python -u -m svm355 scale --transport loopback --ranks 1,2,4,8 --repeats 2 \
  --json gpurun_out/scale_loopback.json > gpurun_out/scale_loopback.txt 2>&1 || { tail -20 gpurun_out/scale_loopback.txt; exit 1; }
cat gpurun_out/scale_loopback.txt
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc_smo_$i -o run -- \
    python3 scripts/fit_once.py > gpurun_out/pmc_smo_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_smo_$i.log; exit 1; }
  echo "pmc pass $i ok"
done
