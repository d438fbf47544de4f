#!/bin/bash
# Round 6: the 1M star cascade (P = 8 rehearsal) with the per-solve choice, each partition Gram released
# after its solve (SVM355_CASCADE_RELEASE_GRAM=1: every rank's pairwise solve then has the whole HBM, as
# on a GPU of its own), against the decomposition everywhere (gpu_r6_n.sh: 2.9 s critical path).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6o
export TMPDIR=/tmp PYTHONUNBUFFERED=1 SVM355_CASCADE_SERIAL_SOLVES=1 SVM355_CASCADE_RELEASE_GRAM=1
timeout -k 10 1000 python -u bench.py --gpus 8 --cascade --topology star --transport loopback --rows 1000000 --test-rows 2000 \
  --steps 1 --warmup 0 --baseline-1gpu 0 --out gpurun_out/r6o/star_auto.json > gpurun_out/r6o/star_auto.log 2>&1 \
  || { tail -20 gpurun_out/r6o/star_auto.log; exit 1; }
python3 - gpurun_out/r6o/star_auto.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: d.get(k) for k in ("critical_path_solve_ms", "rounds", "n_sv", "rank0_smo_iterations", "solver", "ms_per_step", "sv_history", "per_round_critical_path")})
PY
