#!/bin/bash
# Round 5: the inner stop fraction re-checked with the two-pair inner solve.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5w
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/decomp_env_sweep.py 60000,250000 '' 'SVM355_DECOMP_TAU_FRAC=0.03' \
  'SVM355_DECOMP_TAU_FRAC=0.05' 'SVM355_DECOMP_TAU_FRAC=0.15' 'SVM355_DECOMP_TAU_FRAC=0.2' 'SVM355_DECOMP_TAU_FRAC=0.3' \
  > gpurun_out/r5w/sweep.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5w/sweep.txt; exit $rc
