#!/bin/bash
# Round 3 experiment: is the inner solve's row read faster when K(W, W) sits in the XCD's L2?
# SVM355_DECOMP_WARM=1: the inner workgroup reads K(W, W) once at its start (q = 512 / 640: 2 / 3.2 MB).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for q in 512 640; do
  for wm in 0 1; do
    echo "== q $q warm $wm"
    SVM355_DECOMP_WARM=$wm SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 $q 1 noref \
      > gpurun_out/warm_prof_q${q}_w$wm.txt 2>&1 || { tail -20 gpurun_out/warm_prof_q${q}_w$wm.txt; exit 1; }
    grep "decomp prof" gpurun_out/warm_prof_q${q}_w$wm.txt
    SVM355_DECOMP_WARM=$wm timeout -k 10 120 python -u scripts/decomp_timing.py 60000 $q 3 noref \
      > gpurun_out/warm_time_q${q}_w$wm.txt 2>&1 || { tail -20 gpurun_out/warm_time_q${q}_w$wm.txt; exit 1; }
    grep "decomp q" gpurun_out/warm_time_q${q}_w$wm.txt
  done
done
