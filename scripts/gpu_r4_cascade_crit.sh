#!/bin/bash
# 60k cascade critical path on one GPU (P thread-ranks over loopback, every solve timed alone), star and
# tree at P = 2 / 4 / 8, every local / merge solve by the warm-started decomposition and, for comparison,
# by the reference's pairwise SMO.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp SVM355_CASCADE_SERIAL_SOLVES=1
for solver in ${SOLVERS:-auto decomp smo}; do
for topo in star tree; do
  for P in 2 4 8; do
    f=gpurun_out/r4crit_${solver}${WSS:+_$WSS}_${topo}_P$P
    sarg="--solver $solver"; [ "$solver" = auto ] && sarg=""; [ -n "$WSS" ] && sarg="$sarg --wss $WSS"
    timeout -k 10 300 python -u bench.py --gpus $P --cascade $sarg --topology $topo --transport loopback \
      --steps 2 --warmup 1 --baseline-1gpu 0 --out $f.json > $f.log 2>&1 || { tail -20 $f.log; exit 1; }
    python - "$f.json" "$solver $topo P=$P" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keys = ["critical_path_solve_ms", "rounds", "n_sv", "sv_ids_digest", "b", "rank0_smo_iterations", "skipped_solves",
        "accuracy", "solver", "sv_history"]
print(sys.argv[2], json.dumps({k: d.get(k) for k in keys}))
print("   per round:", d.get("per_round_critical_path"))
PY
  done
done
done
