#!/bin/bash
# Counters of the narrow column store at 1M (cache on): one pass per counter block.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
i=0
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  SVM355_DECOMP_CCACHE_FIXED=1 timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex narrow --output-format csv \
    -d gpurun_out/r4npmc$i -o run -- python3 scripts/decomp_cache_timing.py 1000000 > gpurun_out/r4npmc$i.log 2>&1 \
    || { tail -5 gpurun_out/r4npmc$i.log; exit 1; }
done
