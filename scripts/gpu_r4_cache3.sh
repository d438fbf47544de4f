#!/bin/bash
# Round 4: column-cache reader variants (SVM355_DECOMP_CCACHE_RD) at 1M / 250k: fit time, bit identity,
# per-kernel time.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
for v in 0 3 5 6; do
  echo "== RD=$v" >> gpurun_out/r4rd.txt
  SVM355_DECOMP_CCACHE_RD=$v timeout -k 10 300 python -u scripts/decomp_cache_timing.py 1000000 250000 >> gpurun_out/r4rd.txt 2>&1 || exit 1
done
for v in 5 6; do
  SVM355_DECOMP_CCACHE_RD=$v SVM355_DECOMP_CCACHE_FIXED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/r4rdprof$v -o run -- python3 scripts/decomp_cache_timing.py 1000000 > gpurun_out/r4rdprof$v.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r4rd.txt
