#!/bin/bash
# Column-store kernel timing vs the number of columns (1M rows), and the GEMV cache-path unit test.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_decomp_oracle.py -k gemv \
  > gpurun_out/r4cs_pytest.txt 2>&1 || { tail -30 gpurun_out/r4cs_pytest.txt; exit 1; }
for m in 1 8 16 32 64; do
  SVM355_GEMV_VIA_CACHE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4cs_$m -o run \
    -- python3 scripts/colstore_bench.py 1000000 $m > gpurun_out/r4cs_$m.log 2>&1 || { tail -5 gpurun_out/r4cs_$m.log; exit 1; }
done
tail -3 gpurun_out/r4cs_pytest.txt
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d gpurun_out/r4trace -o run \
  -- python3 scripts/trace_demo.py > gpurun_out/r4trace.log 2>&1 || { tail -20 gpurun_out/r4trace.log; exit 1; }
python scripts/trace_summary.py gpurun_out/r4trace > gpurun_out/r4trace_summary.txt 2>&1
cat gpurun_out/r4trace_summary.txt
