#!/bin/bash
# Round 4: the whole GPU test suite (as the driver runs it), smoke(), the 1-GPU bench and the N=2 rehearsal.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r4full_pytest.txt 2>&1 || { tail -40 gpurun_out/r4full_pytest.txt; exit 1; }
tail -3 gpurun_out/r4full_pytest.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4full_smoke.txt 2>&1 \
  || { tail -20 gpurun_out/r4full_smoke.txt; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/r4full_bench1.json > gpurun_out/r4full_bench1.log 2>&1 \
  || { tail -20 gpurun_out/r4full_bench1.log; exit 1; }
python - <<'PY'
import json
a = json.load(open("gpurun_out/r4full_bench1.json"))
print("1 GPU", a["value"], a["iterations"], a["b"], a["n_sv"], a["accuracy"], a.get("f64_input_fit_ms"), a["pairwise_solver"]["fit_ms"])
PY
SOLVERS=auto bash scripts/gpu_r4_cascade_crit.sh > gpurun_out/r4crit3.txt 2>&1 || { tail -5 gpurun_out/r4crit3.txt; exit 1; }
grep -v "per round" gpurun_out/r4crit3.txt
