#!/bin/bash
# Round 3 check D: decomposition inner-workgroup shapes, and where a fresh process's first GPU
# operation pays its one-off cost.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3d_decomp_pytest.txt 2>&1 || { tail -40 gpurun_out/r3d_decomp_pytest.txt; exit 1; }
tail -2 gpurun_out/r3d_decomp_pytest.txt
for nt in 1024 512 256; do
  SVM355_DECOMP_NT=$nt timeout -k 10 200 python -u scripts/decomp_timing.py 60000 1024,512 > gpurun_out/r3d_decomp_nt$nt.txt 2>&1 || \
    { cat gpurun_out/r3d_decomp_nt$nt.txt; exit 1; }
  echo "== NT=$nt"; grep -v amdgpu.ids gpurun_out/r3d_decomp_nt$nt.txt
done
for o in h2d,ctx,native,torch,fit torch,h2d,ctx,native,fit ctx,native,h2d,torch,fit; do
  timeout -k 10 120 python -u scripts/first_op_probe.py $o > gpurun_out/r3d_first_$o.txt 2>&1 || { cat gpurun_out/r3d_first_$o.txt; exit 1; }
  echo "== $o"; grep -v amdgpu.ids gpurun_out/r3d_first_$o.txt
done
