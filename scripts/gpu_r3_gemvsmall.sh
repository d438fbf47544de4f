#!/bin/bash
# Round 3: GEMV grid at small row counts (one GPU's share of the distributed solve: 60k / 8 = 7.5k rows,
# 60k / 2 = 30k): walking (-1) vs one workgroup per half (0), via decomp fits at n = 7.5k / 15k / 30k, and
# the distributed rehearsal at P = 8 (each rank's GEMV covers 7.5k rows); decomp tests under the default.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/small_pytest.txt 2>&1 || { tail -30 gpurun_out/small_pytest.txt; exit 1; }
tail -1 gpurun_out/small_pytest.txt
for n in 7500 15000 30000; do
  for gc in -1 0; do
    SVM355_GEMV_GC=$gc timeout -k 10 120 python -u scripts/decomp_timing.py $n 1024 5 noref > gpurun_out/small_${n}_$gc.txt 2>&1 || { tail -20 gpurun_out/small_${n}_$gc.txt; exit 1; }
    echo "n $n GC $gc: $(grep 'decomp q' gpurun_out/small_${n}_$gc.txt | cut -c1-100)"
  done
done
timeout -k 10 300 python -u bench.py --gpus 8 --transport loopback --steps 3 --warmup 1 --baseline-1gpu 2 \
  --out gpurun_out/small_p8.json > gpurun_out/small_p8.log 2>&1 || { tail -20 gpurun_out/small_p8.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/small_p8.json')); print('rehearsal P=8', d['value'], 'bit_identical', d.get('bit_identical_to_1gpu'), 'single', d.get('single_gpu_s'))"
