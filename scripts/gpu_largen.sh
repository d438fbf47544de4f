#!/bin/bash
# Large-n cascade rehearsal on one GPU: n = 240,000 synthetic MNIST rows, where the
# single-GPU trainer must use the row cache (a 460 GB Gram does not fit in 288 GB).  P = 8 / 4 / 2
# thread-ranks share the GPU over the loopback transport; SVM355_CASCADE_SERIAL_SOLVES=1 makes them
# take turns so every solve is timed alone, and bench.py's critical path (slowest local solve + merge,
# per round) estimates the P-GPU time.  The single-GPU trainer's time is measured in the P = 8 run.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp SVM355_CASCADE_SERIAL_SOLVES=1
N=${N:-240000}
timeout -k 10 500 python -u bench.py --n $N --gpus 8 --transport loopback --steps 1 --warmup 1 --m 2000 \
  --baseline-1gpu 1 --out gpurun_out/largen_P8.json > gpurun_out/largen_P8.log 2>&1 &&
timeout -k 10 500 python -u bench.py --n $N --gpus 4 --transport loopback --steps 1 --warmup 1 --m 2000 \
  --baseline-1gpu 0 --out gpurun_out/largen_P4.json > gpurun_out/largen_P4.log 2>&1 &&
timeout -k 10 600 python -u bench.py --n $N --gpus 2 --transport loopback --steps 1 --warmup 1 --m 2000 \
  --baseline-1gpu 0 --out gpurun_out/largen_P2.json > gpurun_out/largen_P2.log 2>&1; rc=$?
for P in 8 4 2; do
  [ -f gpurun_out/largen_P$P.json ] && python - "$P" <<'PY'
import json, sys
P = sys.argv[1]
d = json.load(open(f"gpurun_out/largen_P{P}.json"))
keys = ["value", "rounds", "n_sv", "critical_path_solve_ms", "critical_path_basis", "per_round_critical_path",
        "rank0_smo_iterations", "max_rank_smo_iterations", "row_cache_solves", "skipped_solves", "single_gpu_s",
        "accuracy", "sv_history", "merged_history", "b"]
print(f"P={P}", json.dumps({k: d.get(k) for k in keys}))
PY
done
exit $rc
