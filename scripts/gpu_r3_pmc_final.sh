#!/bin/bash
# Round 3 (final kernels): PMC counters of the decomposition solver's kernels (f-update GEMV, inner solve, K(W, W)) at 60k:
# two counter passes over one warm fit each (scripts/decomp_timing.py), per-kernel means.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc_gemv2
export TMPDIR=/tmp
R=$(pwd)
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_gemv2/p$i -o p$i -- python3 $R/scripts/decomp_timing.py 60000 1024 1 noref > $R/gpurun_out/pmc_gemv2/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_gemv2/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmc_gemv2/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get('Kernel_Name', '')
        key = 'gemv' if ('igram_tri_kernel' in name and 'true, true' in name) else 'kww' if 'igram_tri_kernel' in name else 'inner' if 'ws_inner' in name else None
        if key is None: continue
        acc[key][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in acc.items():
    print('==', k)
    for c, v in sorted(d.items()):
        print('   %-28s %14.4g (mean over %d dispatches)' % (c, sum(v) / len(v), len(v)))
PY
