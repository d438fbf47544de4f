#!/bin/bash
# Round 3: per-wave candidate picks in the decomposition solver's selection (SVM355_DECOMP_SELW = 1, the
# default when T splits over the 4 waves) vs per-block picks (0): decomp GPU tests, fits at 60k / 250k / 1M.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/selw_pytest.txt 2>&1 || { tail -30 gpurun_out/selw_pytest.txt; exit 1; }
tail -1 gpurun_out/selw_pytest.txt
for sw in 0 1; do
  echo "== selw $sw"
  SVM355_DECOMP_SELW=$sw timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 > gpurun_out/selw_60k_$sw.txt 2>&1 || { tail -20 gpurun_out/selw_60k_$sw.txt; exit 1; }
  grep "decomp q\|smo " gpurun_out/selw_60k_$sw.txt
  SVM355_DECOMP_SELW=$sw timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/selw_250k_$sw.txt 2>&1 || { tail -20 gpurun_out/selw_250k_$sw.txt; exit 1; }
  grep "decomp q" gpurun_out/selw_250k_$sw.txt
  SVM355_DECOMP_SELW=$sw timeout -k 10 200 python -u scripts/decomp_timing.py 1000000 1024 1 noref > gpurun_out/selw_1m_$sw.txt 2>&1 || { tail -20 gpurun_out/selw_1m_$sw.txt; exit 1; }
  grep "decomp q" gpurun_out/selw_1m_$sw.txt
done
