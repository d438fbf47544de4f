#!/bin/bash
# Round 4: the 1-GPU headline, the same fit as a torchrun world-1 rank (the driver's per-process launch),
# and the default N = 2 line rehearsed on the one GPU (with the star / tree cascades after it).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --out gpurun_out/r4d_bench1.json > gpurun_out/r4d_bench1.log 2>&1 \
  || { tail -20 gpurun_out/r4d_bench1.log; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --parallel decomp --steps 10 --warmup 3 --baseline-1gpu 5 --out gpurun_out/r4d_torchrun1.json \
  > gpurun_out/r4d_torchrun1.log 2>&1 || { tail -20 gpurun_out/r4d_torchrun1.log; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 2 --transport loopback --steps 5 --warmup 2 --out gpurun_out/r4d_p2.json \
  > gpurun_out/r4d_p2.log 2>&1 || { tail -20 gpurun_out/r4d_p2.log; exit 1; }
python - <<'PY'
import json
a = json.load(open("gpurun_out/r4d_bench1.json"))
b = json.load(open("gpurun_out/r4d_torchrun1.json"))
c = json.load(open("gpurun_out/r4d_p2.json"))
print("1 GPU", a["value"], "torchrun world 1", b["value"], "speedup_vs_1gpu", b["speedup_vs_1gpu"], "single", b["single_gpu_s"],
      "identical", b["bit_identical_to_1gpu"], "skew", b.get("rccl_skew"), b.get("rccl_runtime"), b.get("rccl_path"))
print("P=2 rehearsal", c["value"], c["config"]["parallelism"], "speedup", c["speedup_vs_1gpu"], "star", c["cascade_star_ms"],
      "tree", c["cascade_tree_ms"], c["cascade_star"]["rounds"], c["cascade_tree"]["rounds"])
PY
