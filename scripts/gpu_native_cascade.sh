#!/bin/bash
# Native cascade (bin/svm_cascade): GPU tests against the Python driver, then 60k runs with the
# loopback transport (P ranks sharing this one GPU) and the RCCL transport on one rank.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "=== tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_cascade.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/native_cascade_tests.txt 2>&1 || { tail -40 gpurun_out/native_cascade_tests.txt; exit 1; }
tail -3 gpurun_out/native_cascade_tests.txt
for cfg in "star 1 rccl" "tree 1 rccl" "star 2 loopback" "star 4 loopback" "star 8 loopback" "tree 8 loopback"; do
  set -- $cfg
  echo "=== 60k $1 P=$2 $3"
  timeout -k 10 300 svm355/bin/svm_cascade --synthetic 60000,10000 --topology $1 --gpus $2 --transport $3 \
    --json gpurun_out/native_$1$2$3.json > gpurun_out/native_$1$2$3.txt 2>&1 || { tail -20 gpurun_out/native_$1$2$3.txt; exit 1; }
  grep -E "Round|Converged|Final|accuracy|time =" gpurun_out/native_$1$2$3.txt | tail -6
done
