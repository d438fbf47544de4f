#!/bin/bash
# Round 5: L2 prefetch helpers for the inner solve's K(W, W) rows -- fit-time sweep at 60k and 250k.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5m
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/decomp_l2_prefetch_probe.py 60000,250000 > gpurun_out/r5m/probe.txt 2>&1
rc=$?; cat gpurun_out/r5m/probe.txt | tail -20; exit $rc
