#!/bin/bash
# One-vs-rest GPU tests (incl. the batched second-order kernel) and the 60k first/second-order A/B.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "ovr" \
  > gpurun_out/t_ovr.txt 2>&1 || { tail -30 gpurun_out/t_ovr.txt; exit 1; }
tail -3 gpurun_out/t_ovr.txt
timeout -k 10 300 python -u scripts/ovr_wss_ab.py > gpurun_out/ovr_wss.txt 2>&1 || { tail -20 gpurun_out/ovr_wss.txt; exit 1; }
grep -v amdgpu gpurun_out/ovr_wss.txt
