#!/bin/bash
# Round 6 final checks: smoke(), the whole GPU suite, the 1-GPU bench, a per-process P = 2 rehearsal.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6l
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6l/smoke.txt 2>&1 || { tail -20 gpurun_out/r6l/smoke.txt; exit 1; }
grep smoke: gpurun_out/r6l/smoke.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/r6l/bench.json > gpurun_out/r6l/bench.log 2>&1 || { tail -20 gpurun_out/r6l/bench.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r6l/bench.json'))
print(d['value'], d['ms_per_step'], 'cold', d['cold_fit_ms'], 'init', d['device_init_ms'], 'f64', d['f64_input_fit_ms'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --parallel decomp --transport hostcomm --steps 3 --warmup 1 > gpurun_out/r6l/hostcomm2.log 2>&1 || { tail -20 gpurun_out/r6l/hostcomm2.log; exit 1; }
grep '"metric"' gpurun_out/r6l/hostcomm2.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['config']['parallelism'], d.get('bit_identical_to_1gpu'), d.get('speedup_vs_1gpu'))"
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r6l/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r6l/pytest.txt; exit $rc
