#!/bin/bash
# Round 6: the distributed decomposition at 1M with the column cache forced on every rank (P = 8: 125k
# rows per rank sit below the 192 MiB threshold, so the ranks recompute by GEMV), warm fits.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6j
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for cc in "" 1; do
  tag=${cc:-default}
  if [ -n "$cc" ]; then export SVM355_DECOMP_CCACHE=$cc; else unset SVM355_DECOMP_CCACHE; fi
  timeout -k 10 500 python3 -u -m svm355 scale --transport loopback --ranks 1,4,8 --sizes 1000000 \
    --test-rows 1000 --repeats 2 --warmup 1 --json gpurun_out/r6j/scale_$tag.json > gpurun_out/r6j/scale_$tag.txt 2>&1 \
    || { tail -20 gpurun_out/r6j/scale_$tag.txt; exit 1; }
  grep -v "amdgpu.ids" gpurun_out/r6j/scale_$tag.txt | tail -6
done
