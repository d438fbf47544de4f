#!/bin/bash
# Round 3: the decomposition inner solve with contiguous per-thread points (thread t holds W[t PER + e];
# its row entries are PER / 2 16-byte loads instead of PER strided 8-byte loads): decomp GPU tests, phase
# profile, fit times at 60k and 250k, bench (the trajectory must be unchanged: b, iterations).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/contig_pytest.txt 2>&1 || { tail -30 gpurun_out/contig_pytest.txt; exit 1; }
tail -1 gpurun_out/contig_pytest.txt
SVM355_DECOMP_PROF=1 timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 1 noref > gpurun_out/contig_prof.txt 2>&1 || { tail -20 gpurun_out/contig_prof.txt; exit 1; }
grep "decomp prof" gpurun_out/contig_prof.txt
for w in 2 1; do
  SVM355_DECOMP_WSS=$w timeout -k 10 120 python -u scripts/decomp_timing.py 60000 1024 5 noref > gpurun_out/contig_time_w$w.txt 2>&1 || { tail -20 gpurun_out/contig_time_w$w.txt; exit 1; }
  grep "decomp q" gpurun_out/contig_time_w$w.txt
done
timeout -k 10 200 python -u scripts/decomp_timing.py 250000 1024 2 noref > gpurun_out/contig_250k.txt 2>&1 || { tail -20 gpurun_out/contig_250k.txt; exit 1; }
grep "decomp q" gpurun_out/contig_250k.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --out gpurun_out/contig_bench.json > gpurun_out/contig_bench.log 2>&1 || { tail -20 gpurun_out/contig_bench.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/contig_bench.json'))
print('bench', d['value'], d['ms_per_step'], 'it', d['iterations'], 'b', d['b'], 'nsv', d['n_sv'], 'acc', d['accuracy'], 'steps', d['step_ms'])"
