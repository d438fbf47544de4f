#!/bin/bash
# Cascade paths on one GPU: bench over RCCL with one rank, a 2-rank gloo rehearsal (both ranks on the card),
# and the cascade GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --cascade --steps 2 --warmup 1 > gpurun_out/casc_nccl1.txt 2>&1 || { tail -30 gpurun_out/casc_nccl1.txt; exit 1; }
grep metric gpurun_out/casc_nccl1.txt | cut -c1-400
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --backend gloo --steps 1 --warmup 1 > gpurun_out/casc_gloo2.txt 2>&1 || { tail -30 gpurun_out/casc_gloo2.txt; exit 1; }
grep metric gpurun_out/casc_gloo2.txt | cut -c1-400
timeout -k 10 300 python -u -m pytest tests/test_gpu_cascade.py tests/test_gpu_kernels.py -k "cascade or svc" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_casc.txt 2>&1; rc=$?; tail -12 gpurun_out/pytest_casc.txt; exit $rc
