#!/bin/bash
# Round 3: atomic-merge decomposition inner solve (SVM355_DECOMP_AT = 1, default) vs the publish + fold
# kernel (0): decomp GPU tests on the new kernel, clock64 phase profiles, warm fit times, 250k / 1M.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/at_pytest.txt 2>&1 || { tail -30 gpurun_out/at_pytest.txt; exit 1; }
tail -1 gpurun_out/at_pytest.txt
for w in 2 1; do
  for at in 0 1; do
    echo "== wss $w at $at"
    SVM355_DECOMP_WSS=$w SVM355_DECOMP_AT=$at SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref \
      > gpurun_out/at_prof_w${w}_a$at.txt 2>&1 || { tail -20 gpurun_out/at_prof_w${w}_a$at.txt; exit 1; }
    grep "decomp prof" gpurun_out/at_prof_w${w}_a$at.txt
    SVM355_DECOMP_WSS=$w SVM355_DECOMP_AT=$at timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024,512 3 \
      > gpurun_out/at_time_w${w}_a$at.txt 2>&1 || { tail -20 gpurun_out/at_time_w${w}_a$at.txt; exit 1; }
    grep "decomp q\|smo " gpurun_out/at_time_w${w}_a$at.txt
  done
done
for at in 0 1; do
  echo "== 250k / 1M at $at"
  SVM355_DECOMP_AT=$at timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/at_250k_a$at.txt 2>&1 || { tail -20 gpurun_out/at_250k_a$at.txt; exit 1; }
  grep "decomp q" gpurun_out/at_250k_a$at.txt
  SVM355_DECOMP_AT=$at timeout -k 10 200 python -u scripts/decomp_timing.py 1000000 1024 1 noref > gpurun_out/at_1m_a$at.txt 2>&1 || { tail -20 gpurun_out/at_1m_a$at.txt; exit 1; }
  grep "decomp q" gpurun_out/at_1m_a$at.txt
done
