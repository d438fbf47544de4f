#!/bin/bash
# Round 5: is the cold upload's extra ~8 ms the first large DMA of the process (copy-engine set-up) or
# the first write into a fresh device allocation?  The upload probe after a 32 MB scratch copy from
# pageable / pinned memory, against none; staging ring off (direct copies).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5g
export TMPDIR=/tmp SVM355_H2D_STAGING=0
for pre in none pageable pinned; do
  PRE=$([ $pre = none ] && echo "" || echo $pre) timeout -k 10 120 python3 scripts/upload_probe.py \
    > gpurun_out/r5g/upload_$pre.txt 2>&1 || exit 1
done
grep -E "^[0-9] |pre-copy" gpurun_out/r5g/upload_*.txt
