#!/bin/bash
# Round 3: candidate-row prefetch in the decomposition inner solve (SVM355_DECOMP_PF = 0 / 1): decomp GPU
# tests with it on, clock64 phase profile, warm fit times (first- and second-order inner j), 250k.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
SVM355_DECOMP_PF=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pf_pytest.txt 2>&1 || { tail -30 gpurun_out/pf_pytest.txt; exit 1; }
tail -1 gpurun_out/pf_pytest.txt
for w in 2 1; do
  for pf in 0 1; do
    echo "== wss $w pf $pf"
    SVM355_DECOMP_WSS=$w SVM355_DECOMP_PF=$pf SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref \
      > gpurun_out/pf_prof_w${w}_p$pf.txt 2>&1 || { tail -20 gpurun_out/pf_prof_w${w}_p$pf.txt; exit 1; }
    grep "decomp prof" gpurun_out/pf_prof_w${w}_p$pf.txt
    SVM355_DECOMP_WSS=$w SVM355_DECOMP_PF=$pf timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024,512 3 noref \
      > gpurun_out/pf_time_w${w}_p$pf.txt 2>&1 || { tail -20 gpurun_out/pf_time_w${w}_p$pf.txt; exit 1; }
    grep "decomp q" gpurun_out/pf_time_w${w}_p$pf.txt
  done
done
for pf in 0 1; do
  echo "== 250k pf $pf"
  SVM355_DECOMP_PF=$pf timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/pf_250k_p$pf.txt 2>&1 || { tail -20 gpurun_out/pf_250k_p$pf.txt; exit 1; }
  grep "decomp q" gpurun_out/pf_250k_p$pf.txt
done
