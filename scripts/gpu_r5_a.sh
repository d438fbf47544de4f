#!/bin/bash
# Round 5, first GPU pass: the per-process (torchrun) distributed decomposition at world > 1 on the one
# GPU over the host-staged gloo transport, the decomposition tests (fault injection
# moved into the solve loop), then the 1-GPU bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_decomp.py -x -v --timeout 400 \
  --timeout-method thread > gpurun_out/r5a_pytest.txt 2>&1 || { tail -60 gpurun_out/r5a_pytest.txt; exit 1; }
tail -3 gpurun_out/r5a_pytest.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --decomp-fits 0 --f64-fits 0 --out gpurun_out/r5a_bench.json \
  > gpurun_out/r5a_bench.log 2>&1 || { tail -20 gpurun_out/r5a_bench.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5a_bench.json"))
print(d["value"], d["iterations"], d["b"], d["n_sv"], d["accuracy"], d["cold_fit_ms"])
PY
