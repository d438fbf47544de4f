#!/bin/bash
# Round 3: the single-GPU CLI and the size sweep with --solver smo | decomp (tests/test_gpu_cli.py), and
# the sweep 10k..60k with the decomposition solver.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_cli.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/cli_pytest.txt 2>&1 || { tail -40 gpurun_out/cli_pytest.txt; exit 1; }
tail -4 gpurun_out/cli_pytest.txt
timeout -k 10 300 python -u -m svm355 sweep --synthetic 60000,10000 --warmup 1 --solver decomp --out gpurun_out/cli_sweep_decomp.json > gpurun_out/cli_sweep_decomp.txt 2>&1 || { tail -20 gpurun_out/cli_sweep_decomp.txt; exit 1; }
cat gpurun_out/cli_sweep_decomp.txt
