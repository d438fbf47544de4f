#!/bin/bash
# Round 5: code objects loaded at context creation (cold fit), the scale CLI's solo-timed distributed
# decomposition rehearsal at 60k and 1M (P = 1, 2, 4, 8 on one GPU), and the per-process hostcomm
# bench lines at P = 2 / 4.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5d
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/cold_fit_decomp_probe.py 60000 > gpurun_out/r5d/cold.log 2>&1 &&
grep -E "^fit|^device" gpurun_out/r5d/cold.log &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_decomp.py -x -v --timeout 300 --timeout-method thread \
  -k "scale_cli or column_cache or rank_failure" > gpurun_out/r5d/pytest.txt 2>&1 &&
tail -2 gpurun_out/r5d/pytest.txt &&
timeout -k 10 600 python -u -m svm355 scale --transport loopback --ranks 1,2,4,8 --sizes 60000,1000000 --test-rows 2000 \
  --repeats 1 --warmup 1 --json gpurun_out/r5d/scale.json > gpurun_out/r5d/scale.txt 2>&1 &&
cat gpurun_out/r5d/scale.txt &&
for P in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $P --master-addr 127.0.0.1 \
    --master-port $((29500 + P)) bench.py --gpus $P --parallel decomp --transport hostcomm --steps 5 --warmup 2 \
    --cascade-steps 1 --out gpurun_out/r5d/hostcomm_p$P.json > gpurun_out/r5d/hostcomm_p$P.log 2>&1 || exit 1
done
echo done
