#!/bin/bash
# Round 3: speculative candidate-row loads in the second-order decomposition inner solve (every wave's
# candidate row loaded before the cross-wave fold; SVM355_DECOMP_SPEC=1) vs loads after the fold (=0):
# decomp GPU tests, phase profile and fit times for both (the trajectory must be unchanged).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/spec_pytest.txt 2>&1 || { tail -30 gpurun_out/spec_pytest.txt; exit 1; }
tail -1 gpurun_out/spec_pytest.txt
for sp in 1 0; do
  echo "== SPEC $sp"
  SVM355_DECOMP_SPEC=$sp SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref > gpurun_out/spec_prof_$sp.txt 2>&1 || { tail -20 gpurun_out/spec_prof_$sp.txt; exit 1; }
  grep "decomp prof" gpurun_out/spec_prof_$sp.txt
  SVM355_DECOMP_SPEC=$sp timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref > gpurun_out/spec_time_$sp.txt 2>&1 || { tail -20 gpurun_out/spec_time_$sp.txt; exit 1; }
  grep "decomp q" gpurun_out/spec_time_$sp.txt
  SVM355_DECOMP_SPEC=$sp timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/spec_250k_$sp.txt 2>&1 || { tail -20 gpurun_out/spec_250k_$sp.txt; exit 1; }
  grep "decomp q" gpurun_out/spec_250k_$sp.txt
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --out gpurun_out/spec_bench.json > gpurun_out/spec_bench.log 2>&1 || { tail -20 gpurun_out/spec_bench.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/spec_bench.json'))
print('bench', d['value'], d['ms_per_step'], 'it', d['iterations'], 'b', d['b'], 'nsv', d['n_sv'], 'acc', d['accuracy'], 'steps', d['step_ms'])"
