#!/bin/bash
# Round 6: the Newton polish with a small free-set cap (cheaper steps) at 60k / 250k.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6k
export TMPDIR=/tmp PYTHONUNBUFFERED=1
N=SVM355_DECOMP_NEWTON=1
timeout -k 10 500 python -u scripts/shrink_sweep.py 60000 '' "$N SVM355_DECOMP_NEWTON_MAX=100" "$N SVM355_DECOMP_NEWTON_MAX=150" \
  "$N SVM355_DECOMP_NEWTON_MAX=200" "$N SVM355_DECOMP_NEWTON_MAX=150 SVM355_DECOMP_NEWTON_REPEAT=1" \
  "$N SVM355_DECOMP_NEWTON_MAX=150 SVM355_DECOMP_NEWTON_EVERY=100 SVM355_DECOMP_NEWTON_REPEAT=1" > gpurun_out/r6k/sweep60k.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r6k/sweep60k.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 500 python -u scripts/shrink_sweep.py 250000 '' "$N SVM355_DECOMP_NEWTON_MAX=150" "$N SVM355_DECOMP_NEWTON_MAX=150 SVM355_DECOMP_NEWTON_REPEAT=1" > gpurun_out/r6k/sweep250k.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r6k/sweep250k.txt; exit $rc
