#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python scripts/cascade_rehearsal.py 60000 ${CFGS:-star:1 star:2 star:4 star:8 tree:8} > gpurun_out/cascade_rehearsal.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/cascade_rehearsal.txt | grep -v "^    r" ; grep -c "^    r" gpurun_out/cascade_rehearsal.txt
exit $rc
