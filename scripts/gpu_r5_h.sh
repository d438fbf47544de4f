#!/bin/bash
# Round 5: the copy engine warmed at context creation (cold fit), the 1-GPU bench, the GPU suites.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5h
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/cold_fit_decomp_probe.py 60000 > gpurun_out/r5h/cold.log 2>&1 &&
grep -E "^fit|^device" gpurun_out/r5h/cold.log | sed 's/ .kcache.*//' &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/r5h/bench.json > gpurun_out/r5h/bench.log 2>&1 &&
python3 -c "
import json; d=json.load(open('gpurun_out/r5h/bench.json'))
print(d['value'], 'cold', d['cold_fit_ms'], 'init', d['device_init_ms'], 'f64', d.get('f64_input_fit_ms'), 'pairwise', d['pairwise_solver']['fit_ms'])" &&
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5h/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r5h/pytest.txt; exit $rc
