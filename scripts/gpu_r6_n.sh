#!/bin/bash
# Round 6: the 1M star cascade (P = 8 rehearsal) with the decomposition for every solve, against the
# per-solve choice of r5 (13.1 s critical path, profiles/r5_cascade_1m_rehearsal.json).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6n
export TMPDIR=/tmp PYTHONUNBUFFERED=1 SVM355_CASCADE_SERIAL_SOLVES=1
timeout -k 10 900 python -u bench.py --gpus 8 --cascade --topology star --transport loopback --rows 1000000 --test-rows 2000 \
  --solver decomp --steps 1 --warmup 0 --baseline-1gpu 0 --out gpurun_out/r6n/star_decomp.json > gpurun_out/r6n/star_decomp.log 2>&1 \
  || { tail -20 gpurun_out/r6n/star_decomp.log; exit 1; }
python3 - gpurun_out/r6n/star_decomp.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: d.get(k) for k in ("critical_path_solve_ms", "rounds", "n_sv", "rank0_smo_iterations", "solver", "ms_per_step", "sv_history", "per_round_critical_path")})
PY
