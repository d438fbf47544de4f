#!/bin/bash
# Round 3 experiment: selection granularity of the decomposition solver (SVM355_DECOMP_NB blocks; T = q / (2 NB)
# picks per block and side): outer / inner iteration counts and fit times at 60k and 250k.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for nb in 16 32 64 128; do
  echo "== NB $nb"
  SVM355_DECOMP_NB=$nb timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 3 noref > gpurun_out/nb_60k_$nb.txt 2>&1 || { tail -20 gpurun_out/nb_60k_$nb.txt; exit 1; }
  grep "decomp q" gpurun_out/nb_60k_$nb.txt
done
for nb in 64 128 256; do
  echo "== 250k NB $nb"
  SVM355_DECOMP_NB=$nb timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/nb_250k_$nb.txt 2>&1 || { tail -20 gpurun_out/nb_250k_$nb.txt; exit 1; }
  grep "decomp q" gpurun_out/nb_250k_$nb.txt
done
