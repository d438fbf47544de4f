#!/bin/bash
# Distributed decomposition at 1M rows, P = 8 rehearsed on one GPU (loopback): per-kernel split per rank.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d1m -o run -- \
  python3 bench.py --gpus 8 --transport loopback --parallel decomp --rows 1000000 --test-rows 2000 --steps 1 --warmup 1 \
  --cascade-steps 0 --baseline-1gpu 1 --out gpurun_out/r4d1m.json > gpurun_out/r4d1m.log 2>&1 || { tail -20 gpurun_out/r4d1m.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4d1m.json"))
print({k: d.get(k) for k in ("value", "speedup_vs_1gpu", "single_gpu_s", "bit_identical_to_1gpu", "rank_ms", "stop_reason")})
PY
