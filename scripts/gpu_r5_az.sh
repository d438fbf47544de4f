#!/bin/bash
# Round 5: the inner stop fraction at 3M rows (store-pass bound: fewer outer iterations may pay there).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5az
export TMPDIR=/tmp
for tf in 0.02 0.05 0.1 0.2; do
  SVM355_DECOMP_TAU_FRAC=$tf timeout -k 10 300 python3 -u scripts/decomp_beyond_2m_probe.py 3000000 \
    > gpurun_out/r5az/tf_$tf.txt 2>&1
  rc=$?; echo "tau_frac $tf"; grep "^fit 1" gpurun_out/r5az/tf_$tf.txt; [ $rc -eq 0 ] || exit $rc
done
