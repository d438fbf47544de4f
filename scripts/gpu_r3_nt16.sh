#!/bin/bash
# Round 3: the inner solve's workgroup size again, now that row entries are 16-byte loads
# (SVM355_DECOMP_NT = 128 / 256 / 512 threads x 8 / 4 / 2 points): fit times and phase profile at 60k.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for nt in 256 512 128; do
  echo "== NT $nt"
  SVM355_DECOMP_NT=$nt SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref > gpurun_out/nt16_prof_$nt.txt 2>&1 || { tail -20 gpurun_out/nt16_prof_$nt.txt; exit 1; }
  grep "decomp prof" gpurun_out/nt16_prof_$nt.txt
  SVM355_DECOMP_NT=$nt timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref > gpurun_out/nt16_time_$nt.txt 2>&1 || { tail -20 gpurun_out/nt16_time_$nt.txt; exit 1; }
  grep "decomp q" gpurun_out/nt16_time_$nt.txt
done
