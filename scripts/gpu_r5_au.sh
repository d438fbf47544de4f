#!/bin/bash
# Round 5: the narrow column store's grid (SVM355_NARROW_WGS_PER_CU) at 1M rows, kernel times by rocprofv3.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5au
export TMPDIR=/tmp
for pc in 0 4 6 8 2; do
  if [ $pc -eq 0 ]; then unset SVM355_NARROW_WGS_PER_CU; else export SVM355_NARROW_WGS_PER_CU=$pc; fi
  PROBE_LABEL="per_cu=$pc" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5au/p$pc -o run \
    --output-format csv -- python3 -u scripts/colstore_probe.py 1000000 1 8 32 64 > gpurun_out/r5au/p$pc.txt 2>&1
  rc=$?; grep "n=" gpurun_out/r5au/p$pc.txt | head -4; [ $rc -eq 0 ] || exit $rc
done
