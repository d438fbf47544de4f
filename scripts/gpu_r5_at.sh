#!/bin/bash
# Round 5: 3M kernel split with the evicting cache (rocprofv3 --kernel-trace), then cache fractions 0.4 / 0.6.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5at
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5at/prof -o run -- \
  python3 -u scripts/decomp_beyond_2m_probe.py 3000000 > gpurun_out/r5at/prof.txt 2>&1
rc=$?; grep "^fit" gpurun_out/r5at/prof.txt; [ $rc -eq 0 ] || exit $rc
for fr in 0.4 0.6; do
  SVM355_DECOMP_CCACHE_FRAC=$fr timeout -k 10 300 python3 -u scripts/decomp_beyond_2m_probe.py 3000000 \
    > gpurun_out/r5at/frac_$fr.txt 2>&1
  rc=$?; echo "frac $fr"; grep "^fit" gpurun_out/r5at/frac_$fr.txt; [ $rc -eq 0 ] || exit $rc
done
