#!/bin/bash
# Round 5: the decomposition past 2,097,152 rows (streamed selection) -- oracle equality of the streamed
# selection kernel, the >2M-row solve, then the decomposition oracle suite and the edge cases again.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5ao
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp_oracle.py tests/test_gpu_edge_cases.py tests/test_gpu_decomp.py \
  -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/r5ao/pytest.txt 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r5ao/pytest.txt | tail -30; exit $rc
