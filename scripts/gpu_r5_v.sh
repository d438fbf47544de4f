#!/bin/bash
# Round 5: inner-solve workgroup shape with the two-pair solve (SVM355_DECOMP_NT 128 / 256 / 512).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5v
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/decomp_env_sweep.py 60000,250000 '' 'SVM355_DECOMP_NT=128' 'SVM355_DECOMP_NT=512' \
  > gpurun_out/r5v/sweep.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5v/sweep.txt; exit $rc
