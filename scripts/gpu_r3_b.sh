#!/bin/bash
# Round 3 check B: the distributed SMO launch forms, the cascade GPU tests after the host-round-trip
# rework, cold-fit probes, and a kernel-trace of the 8-rank loopback cascade (copyBuffer count).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_cascade.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r3b_cascade_pytest.txt 2>&1; rc=$?
tail -8 gpurun_out/r3b_cascade_pytest.txt
[ $rc -eq 0 ] || { grep -B3 -A30 "Error\|FAILED" gpurun_out/r3b_cascade_pytest.txt | head -60; exit $rc; }
bash scripts/gpu_dsmo_launch.sh || exit 1
timeout -k 10 120 python -u scripts/cold_fit_probe.py 60000 fit > gpurun_out/cold_fit.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/cold_fit_probe.py 60000 alloc > gpurun_out/cold_alloc.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/cold_fit.txt gpurun_out/cold_alloc.txt
SVM355_CASCADE_SERIAL_SOLVES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3b_prof_p8 -o run -- \
  python3 bench.py --gpus 8 --transport loopback --parallel cascade --steps 2 --warmup 1 --baseline-1gpu 0 \
  --out gpurun_out/r3b_cascade_p8.json > gpurun_out/r3b_prof_p8.log 2>&1 || { tail -20 gpurun_out/r3b_prof_p8.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3b_cascade_p8.json')); print('cascade p8', d['value'], d['critical_path_solve_ms'], d['rank0_smo_iterations'], d['rank0_phase_ms'])"
f=$(find gpurun_out/r3b_prof_p8 -name "*kernel_stats.csv" | head -1); grep -i "copyBuffer\|Name" "$f" | cut -c1-160
