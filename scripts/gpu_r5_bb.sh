#!/bin/bash
# Round 5: LDS-staged whole-line Q stream in the narrow column store (SVM355_NARROW_STAGE=1, default) against
# the direct fragment loads (=0): the cache's bit-identity tests, kernel times at 1M, then the 1M / 3M fits.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5bb
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp_oracle.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "cache or gemv" > gpurun_out/r5bb/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r5bb/pytest.txt; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  SVM355_NARROW_STAGE=$v PROBE_LABEL=stage$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5bb/s$v \
    -o run --output-format csv -- python3 -u scripts/colstore_probe.py 1000000 1 8 32 > gpurun_out/r5bb/s$v.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  for n in 1000000 3000000; do
    SVM355_NARROW_STAGE=$v timeout -k 10 300 python3 -u scripts/decomp_beyond_2m_probe.py $n > gpurun_out/r5bb/fit_${v}_$n.txt 2>&1
    rc=$?; echo "stage=$v n=$n"; grep "^fit 1" gpurun_out/r5bb/fit_${v}_$n.txt; [ $rc -eq 0 ] || exit $rc
  done
done
