#!/bin/bash
# Two pairs per inner iteration (SVM355_DECOMP_WSS=3, the default) against one (=2): tests, timings, phases.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_decomp_oracle.py \
  tests/test_gpu_decomp.py > gpurun_out/r4dp_pytest.txt 2>&1 || { tail -30 gpurun_out/r4dp_pytest.txt; exit 1; }
tail -2 gpurun_out/r4dp_pytest.txt
for w in 2 3; do
  SVM355_DECOMP_WSS=$w timeout -k 10 300 python -u scripts/decomp_cache_timing.py 60000 250000 1000000 2>&1 | grep -v amdgpu.ids | grep "cache=1\|cache=0" | sed "s/^/wss$w /"
done
SVM355_DECOMP_PROF=1 timeout -k 10 200 python -u scripts/decomp_inner_probe.py 60000 1024 2>&1 | grep -v amdgpu.ids | tail -3
