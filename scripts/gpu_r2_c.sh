#!/bin/bash
# GPU tests (all), record-store scope A/B at 60k, single-GPU bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_all.txt 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu_all.txt
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/pytest_gpu_all.txt | head -80; exit $rc; }
: > gpurun_out/psmo_scope_ab.txt
for v in agent ws agent ws; do
  if [ $v = ws ]; then L=ab_ws/lib; else L=; fi
  echo -n "$v: " >> gpurun_out/psmo_scope_ab.txt
  SVM355_LIB_DIR=$L timeout -k 10 200 python -u scripts/psmo_scope_ab.py 7 2>/dev/null | grep "n=" >> gpurun_out/psmo_scope_ab.txt || exit 1
done
cat gpurun_out/psmo_scope_ab.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench1_r2.txt 2>&1 || { tail gpurun_out/bench1_r2.txt; exit 1; }
cut -c1-400 gpurun_out/bench1_r2.txt | grep metric
