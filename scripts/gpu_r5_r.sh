#!/bin/bash
# Round 5: the driver's 8-rank per-process form rehearsed on one GPU: 8 torchrun processes over gloo
# (hostcomm), 60k distributed decomposition + both cascades.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5r
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 8 --parallel decomp --transport hostcomm --steps 3 --warmup 1 --baseline-1gpu 1 \
  > gpurun_out/r5r/bench8.json 2> gpurun_out/r5r/bench8.err
rc=$?; tail -c 3000 gpurun_out/r5r/bench8.json; tail -n 5 gpurun_out/r5r/bench8.err; exit $rc
