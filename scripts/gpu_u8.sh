set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "u8 or svc_cuda_matches" > gpurun_out/u8_tests.txt 2>&1 && tail -2 gpurun_out/u8_tests.txt &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_u8.txt 2>&1 && cat gpurun_out/bench_u8.txt &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --input f64 > gpurun_out/bench_f64.txt 2>&1 && cat gpurun_out/bench_f64.txt
