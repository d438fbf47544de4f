#!/bin/bash
# Round 5: the cold decomposition fit under a HIP API + kernel trace, and the round-4 exit-time SIGSEGV
# of a profiled single-GPU fit re-run with the crash-evidence handler.  One profiled run; steps chained.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r5c
export TMPDIR=/tmp
export SVM355_CRASH_MAPS=$R/gpurun_out/r5c/crash_{pid}.txt
cd /tmp && timeout -k 10 240 rocprofv3 --runtime-trace --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5c/cold -o run \
  -- python3 $R/scripts/cold_fit_decomp_probe.py 60000 > $R/gpurun_out/r5c/cold.log 2>&1
rc=$?
echo "cold probe under rocprofv3: rc $rc"
grep -E "^fit|^device" $R/gpurun_out/r5c/cold.log
ls $R/gpurun_out/r5c/
exit $rc
