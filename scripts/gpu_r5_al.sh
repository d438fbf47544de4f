#!/bin/bash
# Round 5: NaN-propagating device min/max -- edge cases, the preprocessing kernels' tests, the headline bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5al
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp.py tests/test_gpu_properties.py tests/test_gpu_decomp_oracle.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r5al/pytest.txt 2>&1
rc=$?; tail -n 3 gpurun_out/r5al/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5al/bench.json 2> gpurun_out/r5al/bench.err
rc=$?; python3 -c "import json; d=json.loads(open('gpurun_out/r5al/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['f64_input_fit_ms'], d['n_sv'])"; exit $rc
