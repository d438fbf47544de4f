#!/bin/bash
# Round 5: one-vs-rest with the decomposition solver per class (no Gram) against the batched pairwise solve.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5s
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/ovr_decomp_probe.py 60000 > gpurun_out/r5s/ovr.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5s/ovr.txt | tail -20; exit $rc
