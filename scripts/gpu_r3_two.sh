#!/bin/bash
# Round 3: two-level decomposition inner solve (ws_inner2_kernel, SVM355_DECOMP_INNER = 2, the default) vs
# the one-level kernel (1): decomp GPU tests on it, phase profiles, fit times (TW = 8 / 16 picks per wave
# and side, sub-round stop fraction 0.1 / 0.3) at 60k, 250k and 1M.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/two_pytest.txt 2>&1 || { tail -30 gpurun_out/two_pytest.txt; exit 1; }
tail -1 gpurun_out/two_pytest.txt
SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref > gpurun_out/two_prof.txt 2>&1 || { tail -20 gpurun_out/two_prof.txt; exit 1; }
grep "decomp prof two" gpurun_out/two_prof.txt
for cfg in "1 16 0.1" "2 16 0.1" "2 8 0.1" "2 16 0.3" "2 16 0.03"; do
  set -- $cfg
  echo "== inner $1 tw $2 sfrac $3"
  SVM355_DECOMP_INNER=$1 SVM355_DECOMP_TW=$2 SVM355_DECOMP_SFRAC=$3 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024,512 3 \
    > gpurun_out/two_60k_$1_$2_$3.txt 2>&1 || { tail -20 gpurun_out/two_60k_$1_$2_$3.txt; exit 1; }
  grep "decomp q\|smo " gpurun_out/two_60k_$1_$2_$3.txt
done
for inner in 1 2; do
  echo "== 250k / 1M inner $inner"
  SVM355_DECOMP_INNER=$inner timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/two_250k_$inner.txt 2>&1 || { tail -20 gpurun_out/two_250k_$inner.txt; exit 1; }
  grep "decomp q" gpurun_out/two_250k_$inner.txt
  SVM355_DECOMP_INNER=$inner timeout -k 10 200 python -u scripts/decomp_timing.py 1000000 1024 1 noref > gpurun_out/two_1m_$inner.txt 2>&1 || { tail -20 gpurun_out/two_1m_$inner.txt; exit 1; }
  grep "decomp q" gpurun_out/two_1m_$inner.txt
done
