#!/bin/bash
# Round 4, second GPU pass: the decomposition default everywhere (SVC, CLIs, cascade solves), FP64
# rows, the warm-started cascade, the driver's N > 1 command, then the 1-GPU bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_decomp_oracle.py tests/test_gpu_decomp.py tests/test_gpu_bench.py \
  tests/test_gpu_cascade.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4b_pytest.txt 2>&1 \
  || { tail -60 gpurun_out/r4b_pytest.txt; exit 1; }
tail -3 gpurun_out/r4b_pytest.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --out gpurun_out/r4b_bench.json \
  > gpurun_out/r4b_bench.log 2>&1 || { tail -20 gpurun_out/r4b_bench.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4b_bench.json"))
print(d["value"], d["iterations"], d["b"], d["n_sv"], d["accuracy"], d["timings_ms"].get("outer_iterations"),
      d.get("pairwise_solver", {}).get("fit_ms"), d.get("f64_input_fit_ms"))
PY
