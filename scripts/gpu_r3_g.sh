#!/bin/bash
# Round 3 check G: decomposition tests + inner phase profile + timing per inner shape.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3g_decomp_pytest.txt 2>&1 || { tail -40 gpurun_out/r3g_decomp_pytest.txt; exit 1; }
tail -2 gpurun_out/r3g_decomp_pytest.txt
for nt in 256 512; do
  SVM355_DECOMP_PROF=1 SVM355_DECOMP_NT=$nt timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref \
    > gpurun_out/r3g_prof_nt$nt.txt 2>&1 || { cat gpurun_out/r3g_prof_nt$nt.txt; exit 1; }
  echo "== prof NT=$nt"; grep -v amdgpu.ids gpurun_out/r3g_prof_nt$nt.txt
  SVM355_DECOMP_NT=$nt timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024,512 3 \
    > gpurun_out/r3g_time_nt$nt.txt 2>&1 || { cat gpurun_out/r3g_time_nt$nt.txt; exit 1; }
  echo "== time NT=$nt"; grep -v amdgpu.ids gpurun_out/r3g_time_nt$nt.txt
done
