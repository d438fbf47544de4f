#!/bin/bash
# Round 3: device-driven outer loop of the decomposition solver, SVM355_DECOMP_BATCH outer iterations
# enqueued per host synchronisation (1 = one sync per outer iteration, as before; default 4): decomp GPU
# tests (incl. the distributed rehearsals and a world-1 RCCL rank), fit times, kernel-trace idle gaps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/batch_pytest.txt 2>&1 || { tail -30 gpurun_out/batch_pytest.txt; exit 1; }
tail -1 gpurun_out/batch_pytest.txt
for b in 1 4 8; do
  echo "== batch $b"
  SVM355_DECOMP_BATCH=$b timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref > gpurun_out/batch_60k_$b.txt 2>&1 || { tail -20 gpurun_out/batch_60k_$b.txt; exit 1; }
  grep "decomp q" gpurun_out/batch_60k_$b.txt
  SVM355_DECOMP_BATCH=$b timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/batch_250k_$b.txt 2>&1 || { tail -20 gpurun_out/batch_250k_$b.txt; exit 1; }
  grep "decomp q" gpurun_out/batch_250k_$b.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/batch_trace -o run -- python3 scripts/decomp_timing.py 60000 1024 2 noref > gpurun_out/batch_trace.log 2>&1 || { tail -20 gpurun_out/batch_trace.log; exit 1; }
echo trace ok
