#!/bin/bash
# Large-n cascade rehearsals on one GPU: 8 thread-ranks over the loopback transport, every solve timed
# alone (SVM355_CASCADE_SERIAL_SOLVES=1) with its resident Gram sized before and released after its
# timed region (SVM355_CASCADE_RELEASE_GRAM=1: 8 resident partition Grams do not fit one GPU together),
# against the single-GPU trainer on the same n (persistent row-cache solver beyond ~189k rows).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do date >> gpurun_out/lnc_tick.txt; sleep 50; done ) &  # progress for the silence watchdog
TICK=$!
trap "kill $TICK 2>/dev/null" EXIT
for n in ${NS:-500000 1000000}; do
  SVM355_RC_VERBOSE=1 SVM355_CASCADE_SERIAL_SOLVES=1 SVM355_CASCADE_RELEASE_GRAM=1 timeout -k 10 ${TL:-500} python -u bench.py --gpus 8 \
    --transport loopback --topology ${TOPO:-star} --n $n --m 2000 --steps 1 --warmup 1 --baseline-1gpu 2 --out gpurun_out/lnc_${TOPO:-star}_$n.json \
    > gpurun_out/lnc_${TOPO:-star}_$n.log 2>&1 || { tail -30 gpurun_out/lnc_${TOPO:-star}_$n.log; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/lnc_${TOPO:-star}_$n.json'))
print($n, {k: d.get(k) for k in ['critical_path_solve_ms', 'single_gpu_s', 'rounds', 'n_sv', 'accuracy', 'rank0_smo_iterations', 'row_cache_solves', 'skipped_solves', 'sv_history', 'merged_history']})
print('  per_round', d['per_round_critical_path'])"
done
