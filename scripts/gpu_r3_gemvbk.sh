#!/bin/bash
# Round 3: the decomposition solver's f-update GEMV with BK = 64 vs 128 int8 columns per LDS stage
# (SVM355_GEMV_BK): fit times and the GEMV kernel's time per call at 60k.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for bk in 128 64; do
  echo "== BK $bk"
  SVM355_GEMV_BK=$bk timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref > gpurun_out/gemvbk_$bk.txt 2>&1 || { tail -20 gpurun_out/gemvbk_$bk.txt; exit 1; }
  grep "decomp q" gpurun_out/gemvbk_$bk.txt
  SVM355_GEMV_BK=$bk timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gemvbk_p$bk -o run -- python3 scripts/decomp_timing.py 60000 1024 2 noref > gpurun_out/gemvbk_p$bk.log 2>&1 || { tail -20 gpurun_out/gemvbk_p$bk.log; exit 1; }
  f=$(find gpurun_out/gemvbk_p$bk -name "*kernel_stats.csv" | head -1)
  python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'igram' in r['Name']: print('   ', r['Name'][:60], r['Calls'], 'avg %.1f us' % (float(r['AverageNs']) / 1e3))
"
done
