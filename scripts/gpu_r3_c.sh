#!/bin/bash
# Round 3 check C: decomposition SMO correctness + timing, cold first fit after the no-PyTorch-kernel
# change, and a kernel-trace of one decomposition fit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r3c_decomp_pytest.txt 2>&1; rc=$?
tail -12 gpurun_out/r3c_decomp_pytest.txt
[ $rc -eq 0 ] || { grep -B3 -A30 "Error\|FAILED" gpurun_out/r3c_decomp_pytest.txt | head -80; exit $rc; }
timeout -k 10 200 python -u scripts/decomp_timing.py 60000 1024,512,256 > gpurun_out/r3c_decomp_timing.txt 2>&1 || \
  { cat gpurun_out/r3c_decomp_timing.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r3c_decomp_timing.txt
timeout -k 10 120 python -u scripts/cold_fit_probe.py 60000 fit > gpurun_out/r3c_cold_fit.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3c_cold_fit.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c_prof_decomp -o run -- \
  python3 scripts/decomp_timing.py 60000 1024 > gpurun_out/r3c_prof_decomp.log 2>&1 || { tail -20 gpurun_out/r3c_prof_decomp.log; exit 1; }
f=$(find gpurun_out/r3c_prof_decomp -name "*kernel_stats.csv" | head -1); cut -c1-200 "$f" | head -20
