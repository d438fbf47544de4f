#!/bin/bash
# Round 5: the column cache at 60k / 120k (default off below 192 MB of quantised rows)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5o
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/decomp_env_sweep.py 60000,120000 '' 'SVM355_DECOMP_CCACHE=1' > gpurun_out/r5o/sweep.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5o/sweep.txt | tail -20; exit $rc
