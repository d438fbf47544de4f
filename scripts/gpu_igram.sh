#!/bin/bash
# Integer-Gram validation: kernel tests, then the 60k trainer on both Gram paths, then the bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for g in int fp64; do
  timeout -k 10 300 svm355/bin/svm_gpu --synthetic 60000,10000 --gram $g > gpurun_out/svm_gpu_$g.txt 2>&1 || { cat gpurun_out/svm_gpu_$g.txt; exit 1; }
  cat gpurun_out/svm_gpu_$g.txt
done
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.txt 2>&1; rc=$?
cat gpurun_out/bench1.txt
exit $rc
