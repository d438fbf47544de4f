#!/bin/bash
# Round 5: host-to-device copies of pageable rows through the context's pinned staging ring (A/B against
# the direct copy: cold and warm fits, the 1-GPU bench), then the GPU test files the upload touches.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5e
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/cold_fit_decomp_probe.py 60000 > gpurun_out/r5e/cold_staged.log 2>&1 &&
SVM355_H2D_STAGING=0 timeout -k 10 120 python3 scripts/cold_fit_decomp_probe.py 60000 > gpurun_out/r5e/cold_direct.log 2>&1 &&
grep -E "^fit" gpurun_out/r5e/cold_staged.log gpurun_out/r5e/cold_direct.log | sed 's/{.upload_preprocess_ms.: \([0-9.]*\).*/upload \1/' &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/r5e/bench_staged.json > gpurun_out/r5e/bench_staged.log 2>&1 &&
SVM355_H2D_STAGING=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --decomp-fits 0 --f64-fits 3 \
  --out gpurun_out/r5e/bench_direct.json > gpurun_out/r5e/bench_direct.log 2>&1 &&
python3 - <<'PY' &&
import json
for k in ("staged", "direct"):
    d = json.load(open(f"gpurun_out/r5e/bench_{k}.json"))
    print(k, d["value"], "cold", d["cold_fit_ms"], "f64", d.get("f64_input_fit_ms"), d["warmup_fit_ms"])
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_decomp.py tests/test_gpu_cascade.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r5e/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r5e/pytest.txt; exit $rc
