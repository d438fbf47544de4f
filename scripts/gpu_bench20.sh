#!/bin/bash
# The driver-shaped bench (20 steps, 5 warm-up) after the byte-path GPU tests; median step and the
# host-side remainder of a fit ("other" = fit - upload - alloc - gram - smo).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "byte_path or headline or u8" > gpurun_out/t_bp.txt 2>&1 || { tail -20 gpurun_out/t_bp.txt; exit 1; }
tail -1 gpurun_out/t_bp.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/bench20.json > gpurun_out/bench20.log 2>&1 \
  || { tail -20 gpurun_out/bench20.log; exit 1; }
python - <<'PY'
import json, statistics as s
d = json.load(open("gpurun_out/bench20.json"))
p = d["step_upload_alloc_gram_smo_fit_ms"]
print(d["value"], d["iterations"], d["b"], "median step", s.median(d["step_ms"]),
      "other", round(s.median([x[4] - x[0] - x[1] - x[2] - x[3] for x in p]), 3), "upload", s.median([x[0] for x in p]))
PY
