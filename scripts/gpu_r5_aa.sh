#!/bin/bash
# Round 5: device warm-ups once per device and process -- OvR first / warm fits, the bench's cold fit, the
# thread-rank and OvR GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5aa
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/ovr_decomp_probe.py 60000 > gpurun_out/r5aa/ovr.txt 2>&1
rc=$?; grep -E "fit|agreement" gpurun_out/r5aa/ovr.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5aa/bench.json 2> gpurun_out/r5aa/bench.err
rc=$?; python3 -c "import json; d=json.loads(open('gpurun_out/r5aa/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['cold_fit_ms'], d['device_init_ms'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_decomp.py tests/test_gpu_cascade.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r5aa/pytest.txt 2>&1
rc=$?; tail -n 2 gpurun_out/r5aa/pytest.txt; exit $rc
