#!/bin/bash
# Round 3: lean cross-wave folds in the decomposition inner solve (fold (value, position) only, the
# winner's alpha / f / K(i, j) read from its wave's slot afterwards; tree fold for the second index):
# decomp GPU tests, phase profile, fit times (the trajectory must be unchanged: b, iterations).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/lean_pytest.txt 2>&1 || { tail -30 gpurun_out/lean_pytest.txt; exit 1; }
tail -1 gpurun_out/lean_pytest.txt
SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref > gpurun_out/lean_prof.txt 2>&1 || { tail -20 gpurun_out/lean_prof.txt; exit 1; }
grep "decomp prof" gpurun_out/lean_prof.txt
for w in 2 1; do
  SVM355_DECOMP_WSS=$w timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024,512 5 noref > gpurun_out/lean_time_w$w.txt 2>&1 || { tail -20 gpurun_out/lean_time_w$w.txt; exit 1; }
  grep "decomp q" gpurun_out/lean_time_w$w.txt
done
timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/lean_250k.txt 2>&1 || { tail -20 gpurun_out/lean_250k.txt; exit 1; }
grep "decomp q" gpurun_out/lean_250k.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lean_prof_k -o run -- python3 scripts/decomp_timing.py 60000 1024 3 noref > gpurun_out/lean_prof_k.log 2>&1 || { tail -20 gpurun_out/lean_prof_k.log; exit 1; }
f=$(find gpurun_out/lean_prof_k -name "*kernel_stats.csv" | head -1)
python -c "
import csv
for r in csv.DictReader(open('$f')):
    print('   ', r['Name'][:70].ljust(70), r['Calls'].rjust(6), '%10.3f ms' % (int(r['TotalDurationNs']) / 1e6), '%9.1f us' % (float(r['AverageNs']) / 1e3))
" > gpurun_out/lean_prof_k.txt; head -12 gpurun_out/lean_prof_k.txt
