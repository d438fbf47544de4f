#!/bin/bash
# Distributed-SMO rehearsal on one GPU: tiny smoke cases first (a fault shows on a small case), then
# the GPU tests (trajectory = single-GPU solve), then the 60k timing over P teams vs one GPU.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 90 python -u scripts/dsmo_smoke.py 3000x1,3000x2,6000x8 > gpurun_out/dsmo_smoke.txt 2>&1; rc=$?
cat gpurun_out/dsmo_smoke.txt | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_dsmo.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/dsmo_pytest.txt 2>&1; rc=$?
tail -15 gpurun_out/dsmo_pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/dsmo_timing.py > gpurun_out/dsmo_timing.txt 2>&1; rc=$?
tail -30 gpurun_out/dsmo_timing.txt
exit $rc
