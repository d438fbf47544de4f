#!/bin/bash
# Round 5: narrow column store with the next-tile touch (SVM355_NARROW_TOUCH=1) against without, at 1M rows
# (kernel times by rocprofv3), then the 1M and 3M fits both ways (same model expected).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5av
export TMPDIR=/tmp
for t in 0 1; do
  SVM355_NARROW_TOUCH=$t PROBE_LABEL="touch=$t" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5av/t$t \
    -o run --output-format csv -- python3 -u scripts/colstore_probe.py 1000000 1 8 32 > gpurun_out/r5av/t$t.txt 2>&1
  rc=$?; grep "n=" gpurun_out/r5av/t$t.txt | head -3; [ $rc -eq 0 ] || exit $rc
done
for t in 0 1; do
  for n in 1000000 3000000; do
    SVM355_NARROW_TOUCH=$t timeout -k 10 300 python3 -u scripts/decomp_beyond_2m_probe.py $n > gpurun_out/r5av/fit_${t}_$n.txt 2>&1
    rc=$?; echo "touch=$t n=$n"; grep "^fit" gpurun_out/r5av/fit_${t}_$n.txt; [ $rc -eq 0 ] || exit $rc
  done
done
