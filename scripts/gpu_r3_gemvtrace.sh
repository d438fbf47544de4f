#!/bin/bash
# Round 3: per-call durations of the decomposition solver's f-update GEMV (kernel trace, one 60k fit after
# a warm-up fit), to split its time into a per-launch floor and a per-column part.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gemvtrace -o run -- python3 scripts/decomp_timing.py 60000 1024 1 noref > gpurun_out/gemvtrace.log 2>&1 || { tail -20 gpurun_out/gemvtrace.log; exit 1; }
f=$(find gpurun_out/gemvtrace -name "*kernel_trace.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
names = {}
for r in rows:
    names.setdefault(r['Kernel_Name'][:60], []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in names.items():
    print('%-60s %5d calls  avg %8.1f us' % (k, len(v), sum(v) / len(v)))
g = [v for k, v in names.items() if 'igram' in k and len(v) > 30]
for v in g:
    last = v[-24:]
    print('last fit, per call (us):', ' '.join('%.0f' % x for x in last))
PY
