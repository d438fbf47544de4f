#!/bin/bash
# Headline-size (60k) cascade critical path on one GPU: P = 2 / 4 / 8 thread-ranks over loopback with
# serial solves (each solve timed alone), star and tree, plus the single-GPU trainer.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp SVM355_CASCADE_SERIAL_SOLVES=1
for topo in star tree; do
  for P in 2 4 8; do
    timeout -k 10 300 python -u bench.py --gpus $P --topology $topo --transport loopback --steps 2 --warmup 1 \
      --baseline-1gpu $([ $P = 8 ] && [ $topo = star ] && echo 3 || echo 0) \
      --out gpurun_out/crit60k_${topo}_P$P.json > gpurun_out/crit60k_${topo}_P$P.log 2>&1 || exit $?
    python - "$topo" "$P" <<'PY'
import json, sys
t, P = sys.argv[1:]
d = json.load(open(f"gpurun_out/crit60k_{t}_P{P}.json"))
keys = ["critical_path_solve_ms", "per_round_critical_path", "rounds", "n_sv", "rank0_smo_iterations",
        "skipped_solves", "single_gpu_s", "accuracy", "b"]
print(f"{t} P={P}", json.dumps({k: d.get(k) for k in keys}))
PY
  done
done
