#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -k "smo or persistent" > gpurun_out/pytest_smo.txt 2>&1; rc=$?
tail -5 gpurun_out/pytest_smo.txt
[ $rc -eq 0 ] || exit $rc
PSMO_STAMPS=1 timeout -k 10 600 python scripts/bench_psmo_shapes.py 60000 ${SHAPES:-256x64 512x64 1024x64 512x32 1024x32 256x32} > gpurun_out/psmo_shapes.txt 2>&1; rc=$?
cat gpurun_out/psmo_shapes.txt | grep -v amdgpu.ids
exit $rc
