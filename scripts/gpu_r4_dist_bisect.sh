#!/bin/bash
# Distributed decomposition rehearsals at large n (bisecting a host SIGSEGV seen at 1M, P = 8).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -X faulthandler -u bench.py --transport loopback --parallel decomp --test-rows 2000 --steps 1 \
    --warmup 1 --cascade-steps 0 --baseline-1gpu 1 --out gpurun_out/r4bis_$name.json "$@" > gpurun_out/r4bis_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run p2_250k --gpus 2 --rows 250000 || exit 1
run p8_250k --gpus 8 --rows 250000 || exit 1
run p2_1m --gpus 2 --rows 1000000 || exit 1
run p8_1m --gpus 8 --rows 1000000 || exit 1
