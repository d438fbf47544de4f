#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONPATH=. TMPDIR=/tmp
for nt in 256 65; do
  for prof in 1 0; do
    echo "== NT=$nt PROF=$prof"
    SVM355_DECOMP_PROF=$prof SVM355_DECOMP_NT=$nt timeout -k 10 120 python scripts/decomp_inner_probe.py 60000 384 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
