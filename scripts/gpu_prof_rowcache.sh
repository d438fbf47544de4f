#!/bin/bash
# rocprofv3 kernel stats of the row-cache SMO at n = 250k (Gram does not fit in HBM).
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d /tmp/prof_rc -o rc -- python3 $R/scripts/large_n_demo.py 250000 > $R/gpurun_out/prof_rc_stdout.txt 2>&1) \
  || { tail -20 gpurun_out/prof_rc_stdout.txt; exit 1; }
grep -v amdgpu gpurun_out/prof_rc_stdout.txt | grep -E "^fit|^data|^test"
python3 - <<'PY' | tee gpurun_out/rowcache_kernel_stats.txt
import csv, glob
f = glob.glob('/tmp/prof_rc/*kernel_stats.csv')[0]
for r in csv.DictReader(open(f)):
    name = r['Name'].split('(')[0][-44:]
    print(f"{name:46s} calls {int(r['Calls']):7d} total {int(r['TotalDurationNs'])/1e6:9.2f} ms  avg {float(r['AverageNs'])/1e3:8.2f} us  max {int(r['MaxNs'])/1e3:9.1f} us  {float(r['Percentage']):5.1f} %")
PY
