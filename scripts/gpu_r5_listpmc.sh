#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5list
cd /tmp && timeout -s KILL 60 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/r5list/avail.txt 2>&1; rc=$?
grep -o -E "\b(TCC|TCP|TA|TD)_[A-Z0-9_]+" $GRAFT_REPO_ROOT/gpurun_out/r5list/avail.txt | sort -u | head -150 > $GRAFT_REPO_ROOT/gpurun_out/r5list/names.txt
wc -l $GRAFT_REPO_ROOT/gpurun_out/r5list/names.txt; exit $rc
