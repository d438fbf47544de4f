#!/bin/bash
# Resident-Gram persistent SMO phase stamps at 60k: XCD-local and device-wide exchange (the
# comparison point for the row-cache solver's hit path).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
SVM355_PSMO_STAMP=1 timeout -k 10 120 python -u scripts/psmo_scope_ab.py 2 > gpurun_out/psmo_stamps_xcd.txt 2>&1 &&
SVM355_PSMO_STAMP=1 SVM355_PSMO_XCD=0 timeout -k 10 120 python -u scripts/psmo_scope_ab.py 2 > gpurun_out/psmo_stamps_dev.txt 2>&1; rc=$?
grep -h "stamps\|n=" gpurun_out/psmo_stamps_xcd.txt gpurun_out/psmo_stamps_dev.txt
exit $rc
