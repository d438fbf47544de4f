#!/bin/bash
# Round-2 cascade validation on one GPU: GPU cascade tests, cascade bench at P=1 (RCCL) and loopback
# rehearsals of P=2/4/8 (ranks share the card, host-staged exchanges: NOT multi-GPU times).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_cascade.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_cascade.txt 2>&1; rc=$?
tail -25 gpurun_out/pytest_gpu_cascade.txt
[ $rc -eq 0 ] || exit $rc
for args in "--cascade --steps 3 --warmup 1" "--gpus 2 --transport loopback --steps 2 --warmup 1" \
            "--gpus 4 --transport loopback --steps 2 --warmup 1" "--gpus 8 --transport loopback --steps 1 --warmup 1" \
            "--gpus 8 --topology tree --transport loopback --steps 1 --warmup 1"; do
  echo "=== bench $args"
  timeout -k 10 300 python -u bench.py $args --baseline-1gpu 0 >> gpurun_out/bench_cascade_r2.txt 2>&1 || { tail -30 gpurun_out/bench_cascade_r2.txt; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/bench_cascade_r2.txt"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"]["parallelism"], d["transport"], "ms", d["ms_per_step"], "rounds", d["rounds"], "nsv", d["n_sv"],
              "crit", d["critical_path_solve_ms"], "r0it", d["rank0_smo_iterations"], d["per_round_critical_path"])
PY
