#!/bin/bash
# Session-4 validation: full GPU test suite (verbose, per-test timeout), smoke, bench, persistent-SMO
# stamps and the kernel-row reuse statistic.  Every GPU step has its own time limit; stop at the first
# failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "=== pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_s4.txt 2>&1 || { tail -40 gpurun_out/pytest_gpu_s4.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu_s4.txt
echo "=== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s4.txt 2>&1 \
  || { cat gpurun_out/smoke_s4.txt; exit 1; }
tail -1 gpurun_out/smoke_s4.txt
echo "=== bench"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_s4.txt 2>&1 \
  || { cat gpurun_out/bench_s4.txt; exit 1; }
cat gpurun_out/bench_s4.txt
echo "=== psmo shapes + stamps"
PSMO_STAMPS=1 timeout -k 10 300 python scripts/bench_psmo_shapes.py 60000 512x64 256x64 \
  > gpurun_out/psmo_s4.txt 2>&1 || { cat gpurun_out/psmo_s4.txt; exit 1; }
cat gpurun_out/psmo_s4.txt
echo "=== small-n solvers"
timeout -k 10 300 python scripts/bench_smo_small.py > gpurun_out/smo_small_s4.txt 2>&1 \
  || { cat gpurun_out/smo_small_s4.txt; exit 1; }
cat gpurun_out/smo_small_s4.txt
echo "=== row reuse"
timeout -k 10 300 python scripts/smo_row_reuse.py > gpurun_out/row_reuse_s4.txt 2>&1 \
  || { cat gpurun_out/row_reuse_s4.txt; exit 1; }
cat gpurun_out/row_reuse_s4.txt
