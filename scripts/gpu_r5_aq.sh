#!/bin/bash
# Round 5: 3M rows -- kernel split (rocprofv3 --stats) at the default column-cache cap, then the same fit
# with the cache allowed 60 % of the HBM.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5aq
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5aq/prof -o run -- \
  python3 -u scripts/decomp_beyond_2m_probe.py 3000000 > gpurun_out/r5aq/prof.txt 2>&1
rc=$?; tail -3 gpurun_out/r5aq/prof.txt; [ $rc -eq 0 ] || exit $rc
SVM355_DECOMP_CCACHE_FRAC=0.6 timeout -k 10 300 python3 -u scripts/decomp_beyond_2m_probe.py 3000000 \
  > gpurun_out/r5aq/frac06.txt 2>&1
rc=$?; tail -3 gpurun_out/r5aq/frac06.txt; exit $rc
