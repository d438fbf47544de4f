#!/bin/bash
# Per-phase wall time of the cascade driver (SVM355_CASCADE_PROFILE=1: each phase ends with a sync).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/cascade_phases.txt
: > $out
for args in "--cascade --steps 3 --warmup 1" "--gpus 8 --transport loopback --steps 1 --warmup 1"; do
  for prof in 0 1; do
    echo "=== SVM355_CASCADE_PROFILE=$prof bench $args" >> $out
    SVM355_CASCADE_PROFILE=$prof timeout -k 10 300 python -u bench.py $args --baseline-1gpu 0 >> $out 2>&1 || { tail -30 $out; exit 1; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/cascade_phases.txt"):
    if l.startswith("==="): print(l.strip())
    if l.startswith("{"):
        d = json.loads(l)
        print(" ms/step", d["ms_per_step"], "driver", d["driver_train_ms"], "crit", d["critical_path_solve_ms"], d["rank0_phase_ms"])
PY
