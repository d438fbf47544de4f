#!/bin/bash
# Round 5: working-set size at 60k (the round-4 sweep was at 250k).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5u
export TMPDIR=/tmp
for q in 512 640 768 896 1024; do
  PYTHONPATH=. timeout -k 10 120 python -u scripts/decomp_inner_probe.py 60000 $q >> gpurun_out/r5u/q.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/r5u/q.txt
