#!/bin/bash
# Exact-integer Gram change check: Gram tests, then the bench (Gram ms, b, iterations must be unchanged).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "int_gram or u8 or svc or row_cache or decision or ovr" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_igram.txt 2>&1 || { tail -30 gpurun_out/pytest_igram.txt; exit 1; }
tail -2 gpurun_out/pytest_igram.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_igram.txt 2>&1 || { tail -20 gpurun_out/bench_igram.txt; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_igram.txt").read().strip().splitlines()[-1])
print(d["ms_per_step"], d["b"], d["iterations"], d["n_sv"], [p[2] for p in d["step_upload_alloc_gram_smo_fit_ms"]])
PY
