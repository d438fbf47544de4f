#!/bin/bash
# Round 3: GEMV grid width, repeated: SVM355_GEMV_GC = 1 / 2 / 0 alternated three times at 60k, then 250k
# and the GEMV kernel time per call for gc = 1.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for gc in 1 2 0; do
    SVM355_GEMV_GC=$gc timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref > gpurun_out/gc2_$gc.txt 2>&1 || { tail -20 gpurun_out/gc2_$gc.txt; exit 1; }
    echo "GC $gc round $r: $(grep 'decomp q' gpurun_out/gc2_$gc.txt | cut -c1-60)"
  done
done
for gc in 1 2; do
  SVM355_GEMV_GC=$gc timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/gc2_250_$gc.txt 2>&1 || { tail -20 gpurun_out/gc2_250_$gc.txt; exit 1; }
  echo "GC $gc 250k: $(grep 'decomp q' gpurun_out/gc2_250_$gc.txt | cut -c1-60)"
done
SVM355_GEMV_GC=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gc2_p1 -o run -- python3 scripts/decomp_timing.py 60000 1024 2 noref > gpurun_out/gc2_p1.log 2>&1 || { tail -20 gpurun_out/gc2_p1.log; exit 1; }
f=$(find gpurun_out/gc2_p1 -name "*kernel_stats.csv" | head -1)
python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'igram' in r['Name']: print('    GC 1', r['Name'][:60], r['Calls'], 'avg %.1f us' % (float(r['AverageNs']) / 1e3))
"
