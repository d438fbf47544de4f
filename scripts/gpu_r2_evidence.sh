#!/bin/bash
# Refresh the secondary measurements on one MI355X: the gpu_svm4.sh size sweep (10k..60k), the opt-in
# second-order bench line, and the 1M-row row-cache fit (first and second order).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m svm355 sweep --synthetic 60000,10000 --warmup 1 --out gpurun_out/sweep_r2.json \
  > gpurun_out/sweep_r2.txt 2>&1 || { tail -20 gpurun_out/sweep_r2.txt; exit 1; }
cat gpurun_out/sweep_r2.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --wss second --out gpurun_out/bench_wss2.json \
  > gpurun_out/bench_wss2.log 2>&1 || { tail -20 gpurun_out/bench_wss2.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_wss2.json')); print('bench wss2', d['ms_per_step'], d['iterations'], d['n_sv'], d['b'], d['accuracy'])"
timeout -k 10 600 python -u scripts/large_n_demo.py 1000000 first,second > gpurun_out/largen_1m.txt 2>&1 || { tail -20 gpurun_out/largen_1m.txt; exit 1; }
cat gpurun_out/largen_1m.txt
