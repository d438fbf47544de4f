#!/bin/bash
# Round 3: pipelined warm-start f kernel (SVM355_WARM_U = 8: the previous kernel; 16 / 32: two groups of
# loads in flight): GPU tests that pin warm starts bit for bit, then the kernel's time per call at
# cascade sizes (rocprofv3 --stats over scripts/warm_start_cost.py: n = 3k / 9k / 30k) and warm re-solves.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
SVM355_WARM_U=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_cascade.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/warmf_pytest.txt 2>&1 || { tail -30 gpurun_out/warmf_pytest.txt; exit 1; }
tail -1 gpurun_out/warmf_pytest.txt
for u in 8 16 32; do
  echo "== U $u"
  SVM355_WARM_U=$u TAG=U$u timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/warmf_$u -o run -- python3 scripts/warm_start_cost.py > gpurun_out/warmf_$u.log 2>&1 || { tail -20 gpurun_out/warmf_$u.log; exit 1; }
  grep "warm re-solve" gpurun_out/warmf_$u.log
  f=$(find gpurun_out/warmf_$u -name "*kernel_stats.csv" | head -1)
  python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'warm_f' in r['Name']: print('   ', r['Name'][:60], r['Calls'], 'avg %.1f us' % (float(r['AverageNs']) / 1e3), 'min %.1f max %.1f' % (int(r['MinNs'])/1e3, int(r['MaxNs'])/1e3))
"
done
