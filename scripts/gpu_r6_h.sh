#!/bin/bash
# Round 6: the device-init split (fresh box: first process, second process, runtime trace), the MFMA
# f64 order check, the 1-GPU bench with the new defaults, the whole GPU suite.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6h
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 scripts/init_trace.py > gpurun_out/r6h/init1.log 2>&1 && grep svmd_create gpurun_out/r6h/init1.log &&
timeout -k 10 120 python3 scripts/init_trace.py > gpurun_out/r6h/init2.log 2>&1 && grep svmd_create gpurun_out/r6h/init2.log &&
timeout -k 10 200 rocprofv3 --runtime-trace --kernel-trace -d gpurun_out/r6h/rt -o run -- python3 scripts/init_trace.py > gpurun_out/r6h/init3.log 2>&1 && grep svmd_create gpurun_out/r6h/init3.log &&
python3 scripts/rocpd_api.py gpurun_out/r6h/rt/run_results.db --top 25 --min-ms 2 > gpurun_out/r6h/api.txt 2>&1; tail -5 gpurun_out/r6h/api.txt
timeout -k 10 60 bench_kernels/mfma_f64_order > gpurun_out/r6h/mfma_order.txt 2>&1 && cat gpurun_out/r6h/mfma_order.txt &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/r6h/bench.json > gpurun_out/r6h/bench.log 2>&1 &&
python3 -c "
import json; d=json.load(open('gpurun_out/r6h/bench.json'))
print(d['value'], d['ms_per_step'], 'cold', d['cold_fit_ms'], 'init', d['device_init_ms'])" &&
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r6h/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r6h/pytest.txt; exit $rc
