#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -8 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.txt 2>&1; rc=$?
cat gpurun_out/bench1.txt
[ $rc -eq 0 ] || exit $rc
for n in 2 4; do
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $n --steps 2 --warmup 1 --backend gloo > gpurun_out/bench_gloo$n.txt 2>&1; rc=$?
tail -3 gpurun_out/bench_gloo$n.txt
[ $rc -eq 0 ] || exit $rc
done
