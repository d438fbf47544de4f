#!/bin/bash
# The N > 1 bench lines as the driver will produce them, rehearsed on one GPU:
#  1. torchrun --nproc-per-node 1 bench.py --cascade: the per-process branch (gloo bootstrap,
#     ncclCommInitRank, fit_rank, solve-log gather) with RCCL, at the headline size;
#  2. bench.py --gpus 8 --transport loopback (star, tree): 8 thread-ranks sharing the GPU, every solve
#     timed alone (SVM355_CASCADE_SERIAL_SOLVES=1), so critical_path_solve_ms is the 8-GPU estimate.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 --cascade --steps 5 --warmup 2 --out gpurun_out/reh_torchrun_p1.json \
  > gpurun_out/reh_torchrun_p1.log 2>&1 || { tail -30 gpurun_out/reh_torchrun_p1.log; exit 1; }
echo "torchrun P=1 ok"
for topo in star tree; do
  SVM355_CASCADE_SERIAL_SOLVES=1 timeout -k 10 300 python -u bench.py --gpus 8 --transport loopback --topology $topo \
    --steps 2 --warmup 1 --out gpurun_out/reh_loopback_p8_$topo.json > gpurun_out/reh_loopback_p8_$topo.log 2>&1 \
    || { tail -30 gpurun_out/reh_loopback_p8_$topo.log; exit 1; }
  echo "loopback P=8 $topo ok"
done
python - <<'EOF'
import json
for f in ["reh_torchrun_p1", "reh_loopback_p8_star", "reh_loopback_p8_tree"]:
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, {k: d.get(k) for k in ["value", "n_gpus", "launch", "transport", "rounds", "n_sv", "b", "accuracy",
                                      "critical_path_solve_ms", "rank0_smo_iterations", "single_gpu_s",
                                      "speedup_vs_1gpu", "speedup_vs_ref_cascade_same_P"]})
EOF
