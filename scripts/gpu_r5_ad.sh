#!/bin/bash
# Round 5: the GEMV / column store skip the empty second 32-column tile of a partial half -- oracle and
# numerics tests, the GEMV-per-half probe, the bench.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/r5ad
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_decomp_oracle.py tests/test_gpu_decomp.py tests/test_gpu_properties.py \
  tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ad/pytest.txt 2>&1
rc=$?; tail -n 2 gpurun_out/r5ad/pytest.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/r5ad/prof -o run -- python3 $R/scripts/gemv_halves_probe.py \
  > $R/gpurun_out/r5ad/gemv.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
cd $R && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5ad/bench.json 2> gpurun_out/r5ad/bench.err
rc=$?; python3 -c "import json; d=json.loads(open('gpurun_out/r5ad/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['n_sv'], d['iterations'], d['pairwise_solver']['fit_ms'])"; exit $rc
