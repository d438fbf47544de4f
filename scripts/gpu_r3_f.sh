#!/bin/bash
# Round 3 check F: phase profile of the decomposition inner solve (clock64 stamps), per shape.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for nt in 512 256 1024; do
  for q in 1024 512; do
    SVM355_DECOMP_PROF=1 SVM355_DECOMP_NT=$nt timeout -k 10 120 python -u scripts/decomp_timing.py 60000 $q 1 noref \
      > gpurun_out/r3f_prof_nt${nt}_q$q.txt 2>&1 || { cat gpurun_out/r3f_prof_nt${nt}_q$q.txt; exit 1; }
    echo "== NT=$nt q=$q"; grep -v amdgpu.ids gpurun_out/r3f_prof_nt${nt}_q$q.txt
  done
done
