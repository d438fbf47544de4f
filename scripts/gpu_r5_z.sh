#!/bin/bash
# Round 5: property-based GPU test (random integer data with several range groups).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5z
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_properties.py -m gpu -x -v --timeout 500 --timeout-method thread \
  > gpurun_out/r5z/pytest.txt 2>&1
rc=$?; tail -n 30 gpurun_out/r5z/pytest.txt; exit $rc
