#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/psmo_stamps.py 60000 16 32 64 > gpurun_out/stamps.txt 2>&1; rc=$?
cat gpurun_out/stamps.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_smo_modes.py 60000 > gpurun_out/smo_modes.txt 2>&1; rc=$?
cat gpurun_out/smo_modes.txt
exit $rc
