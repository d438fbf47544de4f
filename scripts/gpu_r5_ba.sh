#!/bin/bash
# Round 5 A/B: nontemporal Q-stream loads in the narrow column store (lib) against the shipped build
# (lib_base, SVM355_LIB_DIR): kernel times at 1M, then the 1M and 3M fits.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5ba
export TMPDIR=/tmp
PKG=parallelizing-support-vector-machine-training-with-gpu-and-mpi_amd
for v in base nt; do
  if [ $v = base ]; then export SVM355_LIB_DIR=$PWD/$PKG/lib_base; else unset SVM355_LIB_DIR; fi
  PROBE_LABEL=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5ba/$v -o run --output-format csv \
    -- python3 -u scripts/colstore_probe.py 1000000 1 8 32 > gpurun_out/r5ba/$v.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  for n in 1000000 3000000; do
    timeout -k 10 300 python3 -u scripts/decomp_beyond_2m_probe.py $n > gpurun_out/r5ba/fit_${v}_$n.txt 2>&1
    rc=$?; echo "$v n=$n"; grep "^fit 1" gpurun_out/r5ba/fit_${v}_$n.txt; [ $rc -eq 0 ] || exit $rc
  done
done
