#!/bin/bash
# Round 6: refresh of the README's sweep and large-n numbers on the round-6 code (defaults).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6p
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -m svm355 sweep --synthetic 60000,10000 --warmup 1 --solver decomp > gpurun_out/r6p/sweep_decomp.txt 2>&1 \
  || { tail -20 gpurun_out/r6p/sweep_decomp.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6p/sweep_decomp.txt
timeout -k 10 300 python3 -m svm355 sweep --synthetic 60000,10000 --warmup 1 --solver smo > gpurun_out/r6p/sweep_smo.txt 2>&1 \
  || { tail -20 gpurun_out/r6p/sweep_smo.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6p/sweep_smo.txt
for s in 2024 0; do
  timeout -k 10 300 python3 -u scripts/fit_decomp_n.py 3000000 2 $s > gpurun_out/r6p/fit3m_seed$s.txt 2>&1 || { tail -20 gpurun_out/r6p/fit3m_seed$s.txt; exit 1; }
  echo "seed $s"; grep -v amdgpu.ids gpurun_out/r6p/fit3m_seed$s.txt
done
