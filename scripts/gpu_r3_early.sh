#!/bin/bash
# Round 3: row i's loads before the inner solve's stop checks (SVM355_DECOMP_EARLY=1) vs after (=0),
# alternated on one box: fit times at 60k (3 rounds x 5 fits each) and 250k.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for e in 1 0; do
    SVM355_DECOMP_EARLY=$e timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref > gpurun_out/early_${e}_$r.txt 2>&1 || { tail -20 gpurun_out/early_${e}_$r.txt; exit 1; }
    echo "EARLY $e round $r: $(grep 'decomp q' gpurun_out/early_${e}_$r.txt)"
  done
done
for e in 1 0; do
  SVM355_DECOMP_EARLY=$e timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/early_250k_$e.txt 2>&1 || { tail -20 gpurun_out/early_250k_$e.txt; exit 1; }
  echo "EARLY $e 250k: $(grep 'decomp q' gpurun_out/early_250k_$e.txt)"
done
