#!/bin/bash
# Full GPU check of the tree: every GPU test, smoke(), bench N=1, and a rocprofv3 kernel-stats profile
# of bench (steps 2, warmup 1).  Outputs under gpurun_out/full_*.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/full_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/full_pytest_gpu.txt
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/full_pytest_gpu.txt | head -80; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.txt 2>&1 || { tail -20 gpurun_out/full_smoke.txt; exit 1; }
tail -1 gpurun_out/full_smoke.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --out gpurun_out/full_bench.json > gpurun_out/full_bench.log 2>&1 || { tail -20 gpurun_out/full_bench.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/full_bench.json')); print('bench', d['value'], d['ms_per_step'], d['iterations'], d['b'], d['n_sv'], d['step_upload_alloc_gram_smo_fit_ms'], 'cold', d.get('cold_fit_ms'), 'init', d.get('device_init_ms'), 'f64', d.get('f64_input_fit_ms'), 'decomp', d.get('decomp_solver'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/full_prof -o run -- python3 bench.py --steps 2 --warmup 1 \
  > gpurun_out/full_prof.log 2>&1 || { tail -20 gpurun_out/full_prof.log; exit 1; }
f=$(find gpurun_out/full_prof -name "*kernel_stats.csv" | head -1); echo "stats: $f"; head -12 "$f" | cut -c1-200
