#!/bin/bash
# Round 6: where shrinking's time goes at 1M (kernel stats on / off) and the active-set trajectory.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SVM355_DECOMP_SHRINK_LOG=1 timeout -k 10 200 python -u scripts/fit_decomp_n.py 1000000 2 > gpurun_out/r6b_log_1m.txt 2>&1 || exit 1
SVM355_DECOMP_SHRINK_LOG=1 timeout -k 10 200 python -u scripts/fit_decomp_n.py 60000 2 > gpurun_out/r6b_log_60k.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b_prof_on -o run -- python3 scripts/fit_decomp_n.py 1000000 2 > gpurun_out/r6b_prof_on.log 2>&1 || exit 1
SVM355_DECOMP_SHRINK=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b_prof_off -o run -- python3 scripts/fit_decomp_n.py 1000000 2 > gpurun_out/r6b_prof_off.log 2>&1 || exit 1
tail -3 gpurun_out/r6b_log_1m.txt gpurun_out/r6b_prof_on.log gpurun_out/r6b_prof_off.log
