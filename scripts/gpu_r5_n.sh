#!/bin/bash
# Round 5: XCD placement of a 1 + 8 H grid, and the inner solve's phase ticks with / without the L2
# prefetch helpers (SVM355_DECOMP_PROF=1: row-load phases are what the helpers would shorten).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5n
export TMPDIR=/tmp
true &&
PYTHONPATH=. SVM355_DECOMP_PROF=1 SVM355_DECOMP_PF_H=0 timeout -k 10 200 python -u scripts/decomp_inner_probe.py 60000 1024 > gpurun_out/r5n/prof_h0.txt 2>&1 &&
PYTHONPATH=. SVM355_DECOMP_PROF=1 SVM355_DECOMP_PF_H=31 timeout -k 10 200 python -u scripts/decomp_inner_probe.py 60000 1024 > gpurun_out/r5n/prof_h31.txt 2>&1 &&
tail -8 gpurun_out/r5n/prof_h0.txt gpurun_out/r5n/prof_h31.txt
