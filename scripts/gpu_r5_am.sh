#!/bin/bash
# Round 5 probe: the f-update GEMV with one workgroup per CU (extra dynamic LDS) -- do the row tiles'
# re-reads across halves then hit the L2?  Kernel trace of the GEMV probe, and the 60k fit, per setting.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r5am
export TMPDIR=/tmp
for pad in 0 60000 0 60000; do
  export SVM355_GEMV_LDS_PAD=$pad
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/r5am/prof_$pad -o run$RANDOM -- python3 $R/scripts/gemv_halves_probe.py \
    > $R/gpurun_out/r5am/gemv_$pad.log 2>&1 || exit $?
  cd $R
done
timeout -k 10 300 python -u scripts/decomp_env_sweep.py 60000 'SVM355_GEMV_LDS_PAD=0' 'SVM355_GEMV_LDS_PAD=60000' 'SVM355_GEMV_LDS_PAD=0' \
  'SVM355_GEMV_LDS_PAD=60000' > gpurun_out/r5am/sweep.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5am/sweep.txt; exit $rc
