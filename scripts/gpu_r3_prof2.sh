#!/bin/bash
# Round 3: second-order j phase split of the decomposition inner solve (clock64 stamps, PROF build)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref > gpurun_out/prof2_q1024.txt 2>&1 || { tail -20 gpurun_out/prof2_q1024.txt; exit 1; }
grep "decomp prof" gpurun_out/prof2_q1024.txt
SVM355_DECOMP_WARM=1 SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 512 1 noref > gpurun_out/prof2_q512_warm.txt 2>&1 || { tail -20 gpurun_out/prof2_q512_warm.txt; exit 1; }
grep "decomp prof" gpurun_out/prof2_q512_warm.txt
