#!/bin/bash
# Round 6: the int8-column bound of the distributed entries; the cascade's warm-started solves with the
# decomposition at other inner stops / shrinking; the per-rank kernel split of the
# distributed decomposition at 1M, P = 4 and 8 (item 2).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6i
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_decomp.py -x -v --timeout 300 --timeout-method thread \
  -k "int8_column_bound" > gpurun_out/r6i/pytest.txt 2>&1 || { tail -40 gpurun_out/r6i/pytest.txt; exit 1; }
tail -2 gpurun_out/r6i/pytest.txt
run() {  # name env... -- bench args
  local name=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env SVM355_CASCADE_SERIAL_SOLVES=1 "${envs[@]}" timeout -k 10 300 python -u bench.py --cascade --transport loopback \
    --steps 2 --warmup 1 --baseline-1gpu 0 --out gpurun_out/r6i/$name.json "$@" > gpurun_out/r6i/$name.log 2>&1 \
    || { tail -20 gpurun_out/r6i/$name.log; return 1; }
  python3 - gpurun_out/r6i/$name.json "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k: d.get(k) for k in ("critical_path_solve_ms", "rounds", "n_sv", "sv_ids_digest", "rank0_smo_iterations", "solver")})
PY
}
for topo in star tree; do
  run auto_$topo -- --gpus 8 --topology $topo &&
  run decomp_$topo -- --gpus 8 --topology $topo --solver decomp &&
  run decomp_tf02_$topo SVM355_DECOMP_TAU_FRAC=0.02 -- --gpus 8 --topology $topo --solver decomp &&
  run decomp_tf0_$topo SVM355_DECOMP_TAU_FRAC=0 -- --gpus 8 --topology $topo --solver decomp &&
  run decomp_shr_$topo SVM355_DECOMP_SHRINK=2 -- --gpus 8 --topology $topo --solver decomp || exit 1
done
for P in 4 8; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r6i/split_P$P -o run -- python3 -m svm355 scale --transport loopback \
    --ranks $P --sizes 1000000 --test-rows 1000 --repeats 1 --warmup 0 > gpurun_out/r6i/split_P$P.log 2>&1 || { tail -20 gpurun_out/r6i/split_P$P.log; exit 1; }
  python3 scripts/rocpd_streams.py gpurun_out/r6i/split_P$P/run_results.db --ranks $P > gpurun_out/r6i/split_P$P.txt 2>&1; head -20 gpurun_out/r6i/split_P$P.txt
done
