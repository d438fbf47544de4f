#!/bin/bash
# Round validation on one MI355X: GPU tests, smoke, 1-GPU bench, RCCL cascade path on one rank,
# 2-rank gloo rehearsal of the multi-GPU bench, CLI sweep.  Every GPU step has its own time limit
# and the script stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.txt 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.txt | tail -${TAILN:-6}; echo "=== $name rc=$rc"; return $rc; }
run pytest_gpu 900 python -m pytest tests -m gpu -x -q || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench1 600 python bench.py --steps 5 --warmup 1 || exit 1
run bench_nccl1_cascade 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 1 --steps 2 --warmup 1 --cascade || exit 1
run bench_gloo2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo || exit 1
run sweep 600 python -m svm355 sweep --synthetic 60000,10000 --warmup 1 || exit 1
