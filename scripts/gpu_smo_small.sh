#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -k "smo or persistent or single" > gpurun_out/pytest_smo.txt 2>&1; rc=$?
tail -5 gpurun_out/pytest_smo.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_smo_small.py > gpurun_out/smo_small.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/smo_small.txt
exit $rc
