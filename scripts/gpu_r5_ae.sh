#!/bin/bash
# Round 5: A/B on one box -- the GEMV with and without the empty-tile skip (SVM355_LIB_DIR = lib_base:
# the build before the change), GEMV-per-half probe under a kernel trace, then the bench, each twice.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r5ae
export TMPDIR=/tmp
for v in base new base new; do
  if [ $v = base ]; then export SVM355_LIB_DIR=$R/svm355/lib_base; else unset SVM355_LIB_DIR; fi
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/r5ae/prof_$v -o run$RANDOM -- python3 $R/scripts/gemv_halves_probe.py \
    > $R/gpurun_out/r5ae/gemv_$v.log 2>&1 || exit $?
  cd $R && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5ae/bench_$v.json 2> gpurun_out/r5ae/bench_$v.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ae/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['pairwise_solver']['fit_ms'])"
done
