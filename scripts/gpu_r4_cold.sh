#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONPATH=. TMPDIR=/tmp SVM355_CASCADE_SERIAL_SOLVES=1
for st in warm cold; do
  for topo in star tree; do
    SVM355_DECOMP_CASCADE_START=$st timeout -k 10 200 python scripts/cascade_solve_log.py 60000 $topo 8 decomp \
      > gpurun_out/r4cold_${st}_${topo}.txt 2>&1 || exit 1
    echo "== start $st: $(grep critical gpurun_out/r4cold_${st}_${topo}.txt)"
  done
done
