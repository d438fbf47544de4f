#!/bin/bash
# Full GPU check of the tree: every GPU test, smoke(), bench N=1 (decomposition headline, pairwise
# alongside), the N > 1 launch forms on one GPU (in-process rehearsal of 2 and 8 ranks; torchrun with one
# rank), and a rocprofv3 kernel-stats profile of bench (steps 2, warmup 1).  Outputs under gpurun_out/full_*.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/full_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/full_pytest_gpu.txt
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/full_pytest_gpu.txt | head -80; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.txt 2>&1 || { tail -20 gpurun_out/full_smoke.txt; exit 1; }
tail -1 gpurun_out/full_smoke.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --out gpurun_out/full_bench.json > gpurun_out/full_bench.log 2>&1 || { tail -20 gpurun_out/full_bench.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/full_bench.json'))
print('bench', d['value'], d['ms_per_step'], d['config']['model'][:40], 'it', d['iterations'], 'b', d['b'], 'nsv', d['n_sv'], 'acc', d['accuracy'])
print('  cold', d.get('cold_fit_ms'), 'init', d.get('device_init_ms'), 'f64', d.get('f64_input_fit_ms'), d.get('f64_input_same_model'))
print('  pairwise', {k: d['pairwise_solver'][k] for k in ('fit_ms', 'same_svs', 'b_minus_headline_b', 'iterations', 'accuracy')})
print('  steps', d['step_ms'])"
for P in 2 8; do
  timeout -k 10 300 python -u bench.py --gpus $P --transport loopback --steps 3 --warmup 1 --baseline-1gpu 2 \
    --out gpurun_out/full_bench_p$P.json > gpurun_out/full_bench_p$P.log 2>&1 || { tail -20 gpurun_out/full_bench_p$P.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/full_bench_p$P.json')); print('rehearsal P=$P', d['config']['parallelism'], d['value'], 'bit_identical', d.get('bit_identical_to_1gpu'), 'single', d.get('single_gpu_s'), 'it', d['iterations'])"
done
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 --parallel decomp --steps 3 --warmup 1 --baseline-1gpu 2 \
  --out gpurun_out/full_bench_torchrun1.json > gpurun_out/full_bench_torchrun1.log 2>&1 || { tail -30 gpurun_out/full_bench_torchrun1.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/full_bench_torchrun1.json')); print('torchrun 1', d['launch'], d['config']['parallelism'], d['value'], 'bit_identical', d.get('bit_identical_to_1gpu'), d.get('rccl_runtime'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/full_prof -o run -- python3 bench.py --steps 2 --warmup 1 \
  > gpurun_out/full_prof.log 2>&1 || { tail -20 gpurun_out/full_prof.log; exit 1; }
f=$(find gpurun_out/full_prof -name "*kernel_stats.csv" | head -1); echo "stats: $f"; head -14 "$f" | cut -c1-160
