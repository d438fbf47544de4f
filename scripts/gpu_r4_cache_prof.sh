#!/bin/bash
# Kernel stats of the decomposition fit with the column cache off and on (argv: n, default 1M).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
N=${1:-1000000}
for c in ${CACHES:-0 1}; do
  SVM355_DECOMP_CCACHE_FIXED=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/r4cprof${c}_$N -o run -- python3 scripts/decomp_cache_timing.py $N > gpurun_out/r4cprof${c}_$N.log 2>&1 \
    || { tail -20 gpurun_out/r4cprof${c}_$N.log; exit 1; }
done
