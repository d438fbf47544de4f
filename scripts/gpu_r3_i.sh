#!/bin/bash
# Round 3 check I: decomposition inner workgroup of 1, 2 or 4 waves (second-order inner selection).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for nt in 256 512; do
  SVM355_DECOMP_NT=$nt SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref \
    > gpurun_out/r3i_prof_nt$nt.txt 2>&1 || { cat gpurun_out/r3i_prof_nt$nt.txt; exit 1; }
  echo "== prof NT=$nt"; grep -v amdgpu.ids gpurun_out/r3i_prof_nt$nt.txt
  SVM355_DECOMP_NT=$nt timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 3 \
    > gpurun_out/r3i_time_nt$nt.txt 2>&1 || { cat gpurun_out/r3i_time_nt$nt.txt; exit 1; }
  echo "== time NT=$nt"; grep -v amdgpu.ids gpurun_out/r3i_time_nt$nt.txt
done
