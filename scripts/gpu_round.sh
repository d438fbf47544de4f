#!/bin/bash
# GPU validation round: GPU tests, smoke, single-GPU bench, rocprof kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "=== $name"; "$@"; local rc=$?; echo "=== $name rc=$rc"; return $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { cat gpurun_out/smoke.txt; exit 1; }
cat gpurun_out/smoke.txt
step bench timeout -k 10 600 python bench.py --steps 3 --warmup 1 --out gpurun_out/bench1.json > gpurun_out/bench1.txt 2>&1 || { cat gpurun_out/bench1.txt; exit 1; }
cat gpurun_out/bench1.txt
