#!/bin/bash
# Round 3: contiguous per-thread positions in the decomposition inner solve (SVM355_DECOMP_CG = 1, the
# default) vs strided (0): decomp GPU tests on the new kernel, phase profiles, fit times at 60k / 250k.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/cg_pytest.txt 2>&1 || { tail -30 gpurun_out/cg_pytest.txt; exit 1; }
tail -1 gpurun_out/cg_pytest.txt
for w in 2 1; do
  for cg in 0 1; do
    echo "== wss $w cg $cg"
    SVM355_DECOMP_WSS=$w SVM355_DECOMP_CG=$cg SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref \
      > gpurun_out/cg_prof_w${w}_c$cg.txt 2>&1 || { tail -20 gpurun_out/cg_prof_w${w}_c$cg.txt; exit 1; }
    grep "decomp prof" gpurun_out/cg_prof_w${w}_c$cg.txt
    SVM355_DECOMP_WSS=$w SVM355_DECOMP_CG=$cg timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref \
      > gpurun_out/cg_time_w${w}_c$cg.txt 2>&1 || { tail -20 gpurun_out/cg_time_w${w}_c$cg.txt; exit 1; }
    grep "decomp q" gpurun_out/cg_time_w${w}_c$cg.txt
  done
done
for cg in 0 1; do
  echo "== 250k cg $cg"
  SVM355_DECOMP_CG=$cg timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/cg_250k_c$cg.txt 2>&1 || { tail -20 gpurun_out/cg_250k_c$cg.txt; exit 1; }
  grep "decomp q" gpurun_out/cg_250k_c$cg.txt
done
