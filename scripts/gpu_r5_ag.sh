#!/bin/bash
# Round 5: 250k / 1M decomposition fits with the final kernels (column cache on by default there).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5ag
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/decomp_env_sweep.py 250000,1000000 '' > gpurun_out/r5ag/sweep.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5ag/sweep.txt; exit $rc
