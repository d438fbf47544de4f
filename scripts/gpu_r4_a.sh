#!/bin/bash
# Round 4, first GPU pass: the decomposition solver's new tests (GEMV unit test, CPU-oracle trajectory,
# warm start), the existing decomposition tests, then the 1-GPU bench (exact division in the inner j
# choice: its cost shows in the fit time).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp_oracle.py tests/test_gpu_decomp.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/r4a_pytest.txt 2>&1 || { tail -40 gpurun_out/r4a_pytest.txt; exit 1; }
tail -3 gpurun_out/r4a_pytest.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --decomp-fits 0 --f64-fits 0 --out gpurun_out/r4a_bench.json \
  > gpurun_out/r4a_bench.log 2>&1 || { tail -20 gpurun_out/r4a_bench.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4a_bench.json"))
print(d["value"], d["iterations"], d["b"], d["n_sv"], d["accuracy"], d["timings_ms"].get("outer_iterations"))
PY
