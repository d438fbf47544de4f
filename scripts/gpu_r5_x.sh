#!/bin/bash
# Round 5 final suite: every GPU test (incl. the 8-process hostcomm bench and the one-vs-rest
# decomposition), then smoke() and the 1-GPU bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5x
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests/ -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r5x/pytest.txt 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5x/pytest.txt | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5x/smoke.txt 2>&1
rc=$?; tail -n 3 gpurun_out/r5x/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r5x/bench.json 2> gpurun_out/r5x/bench.err
rc=$?; tail -c 300 gpurun_out/r5x/bench.json; exit $rc
