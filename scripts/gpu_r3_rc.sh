#!/bin/bash
# Round 3: LDS row cache in the decomposition inner solve (SVM355_DECOMP_RC = 0 / 8 / 16 rows):
# decomp GPU tests with the cache on, then clock64 phase profile + hit rate and warm fit times, inner
# first- and second-order j.  Same b / iteration counts across RC = bit-identical trajectories.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
SVM355_DECOMP_RC=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/rc_pytest.txt 2>&1 || { tail -30 gpurun_out/rc_pytest.txt; exit 1; }
tail -1 gpurun_out/rc_pytest.txt
for w in 2 1; do
  for rc in 0 8 16; do
    echo "== wss $w rc $rc"
    SVM355_DECOMP_WSS=$w SVM355_DECOMP_RC=$rc SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref \
      > gpurun_out/rc_prof_w${w}_r$rc.txt 2>&1 || { tail -20 gpurun_out/rc_prof_w${w}_r$rc.txt; exit 1; }
    grep "decomp prof" gpurun_out/rc_prof_w${w}_r$rc.txt
    SVM355_DECOMP_WSS=$w SVM355_DECOMP_RC=$rc timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 3 noref \
      > gpurun_out/rc_time_w${w}_r$rc.txt 2>&1 || { tail -20 gpurun_out/rc_time_w${w}_r$rc.txt; exit 1; }
    grep "decomp q" gpurun_out/rc_time_w${w}_r$rc.txt
  done
done
for rc in 0 16; do
  echo "== 250k rc $rc"
  SVM355_DECOMP_RC=$rc timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/rc_250k_r$rc.txt 2>&1 || { tail -20 gpurun_out/rc_250k_r$rc.txt; exit 1; }
  grep "decomp q" gpurun_out/rc_250k_r$rc.txt
done
