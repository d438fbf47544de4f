#!/bin/bash
# Round 3: GEMV grid of one workgroup per row tile walking every 64-column half (SVM355_GEMV_GC=-1) vs
# the default (gc = 1: two workgroups per row tile): decomp tests under -1, then alternated fit times at
# 60k, 250k, and the GEMV time per call.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
SVM355_GEMV_GC=-1 timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/walk_pytest.txt 2>&1 || { tail -30 gpurun_out/walk_pytest.txt; exit 1; }
tail -1 gpurun_out/walk_pytest.txt
for r in 1 2 3; do
  for gc in 1 -1; do
    SVM355_GEMV_GC=$gc timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref > gpurun_out/walk_$gc.txt 2>&1 || { tail -20 gpurun_out/walk_$gc.txt; exit 1; }
    echo "GC $gc round $r: $(grep 'decomp q' gpurun_out/walk_$gc.txt | cut -c1-60)"
  done
done
for gc in 1 -1; do
  SVM355_GEMV_GC=$gc timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/walk_250_$gc.txt 2>&1 || { tail -20 gpurun_out/walk_250_$gc.txt; exit 1; }
  echo "GC $gc 250k: $(grep 'decomp q' gpurun_out/walk_250_$gc.txt | cut -c1-60)"
done
SVM355_GEMV_GC=-1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/walk_p -o run -- python3 scripts/decomp_timing.py 60000 1024 2 noref > gpurun_out/walk_p.log 2>&1 || { tail -20 gpurun_out/walk_p.log; exit 1; }
f=$(find gpurun_out/walk_p -name "*kernel_stats.csv" | head -1)
python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'igram' in r['Name']: print('    GC -1', r['Name'][:60], r['Calls'], 'avg %.1f us' % (float(r['AverageNs']) / 1e3))
"
