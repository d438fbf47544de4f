#!/bin/bash
# Round 5: OvR probe twice in separate processes (variance check).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5ab
export TMPDIR=/tmp
for k in 1; do
  timeout -k 10 300 python -u scripts/ovr_workers_probe.py > gpurun_out/r5ab/ovr$k.txt 2>&1 || exit $?
  grep workers gpurun_out/r5ab/ovr$k.txt
done
