#!/bin/bash
# The distributed SMO's launch forms on one GPU: bench.py direct launch (8 teams in one launch),
# torchrun with one process (the per-process path: IPC handles over the store), and two processes
# on the same GPU (IPC between processes, kernels of both running at once).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u bench.py --gpus 8 --transport loopback --parallel smo --steps 5 --warmup 2 \
  --out gpurun_out/dsmo_bench_reh8.json > gpurun_out/dsmo_bench_reh8.log 2>&1 || { tail -20 gpurun_out/dsmo_bench_reh8.log; exit 1; }
cut -c1-1500 gpurun_out/dsmo_bench_reh8.json
timeout -k 10 120 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 --parallel smo --steps 3 --warmup 1 --baseline-1gpu 1 \
  --out gpurun_out/dsmo_bench_torchrun1.json > gpurun_out/dsmo_bench_torchrun1.log 2>&1 || { tail -20 gpurun_out/dsmo_bench_torchrun1.log; exit 1; }
cut -c1-1500 gpurun_out/dsmo_bench_torchrun1.json
timeout -k 10 180 python -u bench.py --gpus 4 --transport loopback --steps 3 --warmup 1 --baseline-1gpu 1 \
  --out gpurun_out/dsmo_bench_auto4.json > gpurun_out/dsmo_bench_auto4.log 2>&1 || { tail -20 gpurun_out/dsmo_bench_auto4.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/dsmo_bench_auto4.json')); print('auto4', d['config']['parallelism'], d['value'], d.get('auto_selection'), d.get('bit_identical_to_1gpu'), d.get('rccl_runtime'), d.get('rccl_path'))"
timeout -k 10 150 python -u scripts/dsmo_procs.py --world 2 --n 3000 > gpurun_out/dsmo_procs2.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dsmo_procs2.txt | tail -12
exit $rc
