#!/bin/bash
# PMC counters of the 60k headline fit's kernels: one rocprofv3 pass per counter block.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r4pmc$i -o run -- \
    python3 bench.py --steps 3 --warmup 2 --decomp-fits 0 --f64-fits 0 > gpurun_out/r4pmc$i.log 2>&1 || { tail -5 gpurun_out/r4pmc$i.log; exit 1; }
done
