#!/bin/bash
# Round 3: the decomposition GEMV grid sized to gc 128-column tiles per row tile, its workgroups walking
# further column halves up to the device-side count (SVM355_GEMV_GC; 0 = one workgroup per half of all
# 1,024 possible columns, most exiting at once): decomp tests, fit times, GEMV time per call.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gc_pytest.txt 2>&1 || { tail -30 gpurun_out/gc_pytest.txt; exit 1; }
tail -1 gpurun_out/gc_pytest.txt
for gc in 2 0 1 4 2 0; do
  SVM355_GEMV_GC=$gc timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref > gpurun_out/gc_$gc.txt 2>&1 || { tail -20 gpurun_out/gc_$gc.txt; exit 1; }
  echo "GC $gc: $(grep 'decomp q' gpurun_out/gc_$gc.txt | cut -c1-120)"
done
for gc in 2 0; do
  SVM355_GEMV_GC=$gc timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/gc250_$gc.txt 2>&1 || { tail -20 gpurun_out/gc250_$gc.txt; exit 1; }
  echo "GC $gc 250k: $(grep 'decomp q' gpurun_out/gc250_$gc.txt | cut -c1-120)"
  SVM355_GEMV_GC=$gc timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gc_p$gc -o run -- python3 scripts/decomp_timing.py 60000 1024 2 noref > gpurun_out/gc_p$gc.log 2>&1 || { tail -20 gpurun_out/gc_p$gc.log; exit 1; }
  f=$(find gpurun_out/gc_p$gc -name "*kernel_stats.csv" | head -1)
  python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'igram' in r['Name']: print('    GC $gc', r['Name'][:60], r['Calls'], 'avg %.1f us' % (float(r['AverageNs']) / 1e3))
"
done
