#!/bin/bash
# Round 3: the inner solve's relative stop (W's gap <= max(2 tau, 2 tau_frac gap); SVM355_DECOMP_TAU_FRAC)
# re-checked on the current kernels: fit time, outer / inner iterations at 60k and 250k.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for tf in 0.1 0.05 0.2 0.3 0.5; do
  SVM355_DECOMP_TAU_FRAC=$tf timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref > gpurun_out/tf_$tf.txt 2>&1 || { tail -20 gpurun_out/tf_$tf.txt; exit 1; }
  echo "tau_frac $tf 60k: $(grep 'decomp q' gpurun_out/tf_$tf.txt | cut -c1-175)"
done
for tf in 0.1 0.2 0.3; do
  SVM355_DECOMP_TAU_FRAC=$tf timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/tf250_$tf.txt 2>&1 || { tail -20 gpurun_out/tf250_$tf.txt; exit 1; }
  echo "tau_frac $tf 250k: $(grep 'decomp q' gpurun_out/tf250_$tf.txt | cut -c1-175)"
done
