#!/bin/bash
# Round 3 check K: bench --parallel decomp launch forms (thread-rank rehearsal, torchrun rank) and the
# kernel split of one-GPU decomposition fits at 250k and 1M (which parts a distributed solve divides).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gpus 4 --transport loopback --parallel decomp --steps 2 --warmup 1 \
  --baseline-1gpu 2 --out gpurun_out/r3k_bench_decomp_p4_rehearsal.json > gpurun_out/r3k_bench_decomp_p4.log 2>&1 || \
  { tail -30 gpurun_out/r3k_bench_decomp_p4.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3k_bench_decomp_p4_rehearsal.json')); print({k: d[k] for k in ('value','ms_per_step','iterations','b','n_sv','bit_identical_to_1gpu','single_gpu_s','accuracy','rank_ms','decomp_stats')})"
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 1 --parallel decomp --steps 2 --warmup 1 --baseline-1gpu 2 \
  --out gpurun_out/r3k_bench_decomp_torchrun1.json > gpurun_out/r3k_bench_decomp_torchrun1.log 2>&1 || \
  { tail -30 gpurun_out/r3k_bench_decomp_torchrun1.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3k_bench_decomp_torchrun1.json')); print({k: d[k] for k in ('value','ms_per_step','iterations','bit_identical_to_1gpu','single_gpu_s','launch','launch_form')})"
for n in 250000 1000000; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3k_prof_$n -o run -- \
    python3 scripts/decomp_timing.py $n 1024 2 noref > gpurun_out/r3k_prof_$n.log 2>&1 || { tail -20 gpurun_out/r3k_prof_$n.log; exit 1; }
  grep -v amdgpu gpurun_out/r3k_prof_$n.log | tail -2
  f=$(find gpurun_out/r3k_prof_$n -name "*kernel_stats.csv" | head -1)
  python -c "
import csv
for r in csv.DictReader(open('$f')):
    print('   ', r['Name'][:70].ljust(70), r['Calls'].rjust(6), '%10.3f ms' % (int(r['TotalDurationNs']) / 1e6))
" | head -14
done
