#!/bin/bash
# Round 5: the distributed decomposition's per-outer-iteration host wait -- the
# world-1 RCCL rank under torchrun against the plain fit (speedup_vs_1gpu), and the per-rank host wait
# of the 8-rank loopback rehearsal at 60k.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5j
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 1 --parallel decomp --steps 20 --warmup 5 --baseline-1gpu 5 --cascade-steps 0 \
  --out gpurun_out/r5j/torchrun1.json > gpurun_out/r5j/torchrun1.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 8 --transport loopback --parallel decomp --steps 3 --warmup 1 \
  --baseline-1gpu 1 --cascade-steps 0 --out gpurun_out/r5j/loopback8.json > gpurun_out/r5j/loopback8.log 2>&1 &&
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r5j/torchrun1.json"))
print("torchrun world 1 (RCCL):", d["value"], "single", d["single_gpu_s"], "speedup_vs_1gpu", d["speedup_vs_1gpu"],
      "bit", d["bit_identical_to_1gpu"], "host wait", d.get("rank_host_wait_ms"), d["rccl_runtime"])
d = json.load(open("gpurun_out/r5j/loopback8.json"))
print("loopback 8:", d["value"], "bit", d["bit_identical_to_1gpu"], "host wait", d.get("rank_host_wait_ms"))
PY
