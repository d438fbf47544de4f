#!/bin/bash
# Round 3 check H: decomposition inner selection first vs second order (60k, 250k), phase profile.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3h_decomp_pytest.txt 2>&1 || { tail -40 gpurun_out/r3h_decomp_pytest.txt; exit 1; }
tail -2 gpurun_out/r3h_decomp_pytest.txt
SVM355_DECOMP_WSS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3h_decomp_pytest_w2.txt 2>&1 || { tail -40 gpurun_out/r3h_decomp_pytest_w2.txt; exit 1; }
tail -2 gpurun_out/r3h_decomp_pytest_w2.txt
for w in 1 2; do
  SVM355_DECOMP_WSS=$w SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024,512 1 noref \
    > gpurun_out/r3h_prof_w$w.txt 2>&1 || { cat gpurun_out/r3h_prof_w$w.txt; exit 1; }
  echo "== prof wss=$w"; grep -v amdgpu.ids gpurun_out/r3h_prof_w$w.txt
  SVM355_DECOMP_WSS=$w timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024,512,256 3 \
    > gpurun_out/r3h_time_w$w.txt 2>&1 || { cat gpurun_out/r3h_time_w$w.txt; exit 1; }
  echo "== time wss=$w"; grep -v amdgpu.ids gpurun_out/r3h_time_w$w.txt
  SVM355_DECOMP_WSS=$w timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref \
    > gpurun_out/r3h_250k_w$w.txt 2>&1 || { cat gpurun_out/r3h_250k_w$w.txt; exit 1; }
  echo "== 250k wss=$w"; grep -v amdgpu.ids gpurun_out/r3h_250k_w$w.txt
done
