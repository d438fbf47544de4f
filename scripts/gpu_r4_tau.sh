#!/bin/bash
# Inner stop fraction (SVM355_DECOMP_TAU_FRAC) with two pairs per inner iteration: fit time per value.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
SVM355_TIMING_VAR=SVM355_DECOMP_TAU_FRAC SVM355_TIMING_VALUES=${VALS:-0.03,0.06,0.1,0.15,0.2,0.3} \
  timeout -k 10 400 python -u scripts/decomp_cache_timing.py ${SIZES:-60000 250000} 2>&1 | grep -v amdgpu.ids | grep "cache="
