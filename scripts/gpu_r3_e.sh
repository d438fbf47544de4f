#!/bin/bash
# Round 3 check E: decomposition SMO with compacted f-update columns: tests, the inner stop fraction
# at 60k, and large n against the row-cache pairwise solve.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3e_decomp_pytest.txt 2>&1 || { tail -40 gpurun_out/r3e_decomp_pytest.txt; exit 1; }
tail -2 gpurun_out/r3e_decomp_pytest.txt
for tf in 0.1 0.05 0.2 0.3; do
  SVM355_DECOMP_TAU_FRAC=$tf timeout -k 10 200 python -u scripts/decomp_timing.py 60000 1024,512 3 > gpurun_out/r3e_tf$tf.txt 2>&1 || \
    { cat gpurun_out/r3e_tf$tf.txt; exit 1; }
  echo "== tau_frac=$tf"; grep -v amdgpu.ids gpurun_out/r3e_tf$tf.txt
done
timeout -k 10 300 python -u scripts/decomp_timing.py 250000 1024 1 > gpurun_out/r3e_250k.txt 2>&1 || { cat gpurun_out/r3e_250k.txt; exit 1; }
echo "== 250k"; grep -v amdgpu.ids gpurun_out/r3e_250k.txt
timeout -k 10 300 python -u scripts/decomp_timing.py 1000000 1024 1 noref > gpurun_out/r3e_1m.txt 2>&1 || { cat gpurun_out/r3e_1m.txt; exit 1; }
echo "== 1M"; grep -v amdgpu.ids gpurun_out/r3e_1m.txt
