#!/bin/bash
# Round 5: column-cache CLOCK eviction -- oracle / bit-identity tests with small caches, then the 3M fit
# with eviction (default) and fill-only (SVM355_DECOMP_CCACHE_EVICT=0), and 1M as a control.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5ar
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp_oracle.py tests/test_gpu_decomp.py -m gpu -v -x \
  --timeout 300 --timeout-method thread > gpurun_out/r5ar/pytest.txt 2>&1
rc=$?; grep -E "cache|passed|failed|^E " gpurun_out/r5ar/pytest.txt | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/decomp_beyond_2m_probe.py 3000000 > gpurun_out/r5ar/evict_3m.txt 2>&1
rc=$?; tail -2 gpurun_out/r5ar/evict_3m.txt; [ $rc -eq 0 ] || exit $rc
SVM355_DECOMP_CCACHE_EVICT=0 timeout -k 10 300 python3 -u scripts/decomp_beyond_2m_probe.py 3000000 \
  > gpurun_out/r5ar/fill_3m.txt 2>&1
rc=$?; tail -2 gpurun_out/r5ar/fill_3m.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/decomp_beyond_2m_probe.py 1000000 > gpurun_out/r5ar/evict_1m.txt 2>&1
rc=$?; tail -2 gpurun_out/r5ar/evict_1m.txt; [ $rc -eq 0 ] || exit $rc
SVM355_DECOMP_CCACHE_EVICT=0 timeout -k 10 300 python3 -u scripts/decomp_beyond_2m_probe.py 1000000 \
  > gpurun_out/r5ar/fill_1m.txt 2>&1
rc=$?; tail -2 gpurun_out/r5ar/fill_1m.txt; exit $rc
