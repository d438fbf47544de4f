#!/bin/bash
# Round 5: the per-process distributed decomposition at a world that does not divide 8 (P = 3, hostcomm on
# one GPU): it must converge (its block partition differs from one GPU's, so bit identity is not expected).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5ah
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=3 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 3 --parallel decomp --transport hostcomm --steps 2 --warmup 1 --baseline-1gpu 1 --cascade-steps 1 \
  > gpurun_out/r5ah/bench3.json 2> gpurun_out/r5ah/bench3.err
rc=$?; python3 -c "
import json; d=json.loads(open('gpurun_out/r5ah/bench3.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('n_gpus','ms_per_step','stop_reason','n_sv','fallback_reason')}); print('star', str(d.get('cascade_star'))[:300]); print('tree', str(d.get('cascade_tree'))[:300])
"; tail -n 3 gpurun_out/r5ah/bench3.err; exit $rc
