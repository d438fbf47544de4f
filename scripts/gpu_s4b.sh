#!/bin/bash
# Session-4 measurements: 1-GPU bench (with prediction time), the 10k->60k size sweep, a rocprofv3
# kernel-trace of the bench, the cascade path over RCCL on one rank, and a 4-rank gloo rehearsal of
# the multi-rank bench path (ranks share the one GPU).  Every GPU step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "=== bench"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_s4b.txt 2>&1 \
  || { cat gpurun_out/bench_s4b.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_s4b.txt
echo "=== sweep"
timeout -k 10 600 python -m svm355 sweep --synthetic 60000,10000 --warmup 1 > gpurun_out/sweep_s4b.txt 2>&1 \
  || { cat gpurun_out/sweep_s4b.txt; exit 1; }
cat gpurun_out/sweep_s4b.txt
echo "=== rocprof bench"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv \
  -d $R/gpurun_out/prof_s4b -o bench -- python3 $R/bench.py --steps 2 --warmup 1 \
  > $R/gpurun_out/prof_s4b_stdout.txt 2>&1) || { tail -20 gpurun_out/prof_s4b_stdout.txt; exit 1; }
find gpurun_out/prof_s4b -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_s4b.csv
find gpurun_out/prof_s4b -name "*marker_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/marker_stats_s4b.csv
head -12 gpurun_out/kernel_stats_s4b.csv
echo "=== cascade over RCCL, 1 rank"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 1 --cascade --steps 2 --warmup 1 > gpurun_out/bench_nccl1_s4b.txt 2>&1 \
  || { tail -30 gpurun_out/bench_nccl1_s4b.txt; exit 1; }
grep metric gpurun_out/bench_nccl1_s4b.txt
echo "=== 4-rank gloo rehearsal (ranks share the GPU)"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29612 bench.py --gpus 4 --backend gloo --steps 1 --warmup 1 > gpurun_out/bench_gloo4_s4b.txt 2>&1 \
  || { tail -30 gpurun_out/bench_gloo4_s4b.txt; exit 1; }
grep metric gpurun_out/bench_gloo4_s4b.txt
