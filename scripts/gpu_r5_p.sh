#!/bin/bash
# Round 5 final pass: the whole GPU suite, the 1-GPU bench (20 steps) and a kernel-trace profile of it.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r5p
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5p/pytest.txt 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5p/pytest.txt | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5p/bench.json 2> gpurun_out/r5p/bench.err
rc=$?; tail -c 400 gpurun_out/r5p/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5p/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 \
  > $R/gpurun_out/r5p/prof.log 2>&1
rc=$?; echo "rocprof rc $rc"; exit $rc
