// Microbenchmark: sustained v_mfma_f64_16x16x4_f64 rate (independent accumulators, all CUs).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k(double* out, int iters, double a0, double b0) {
  f64x4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = f64x4{0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  double s = 0;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  double* out;
  hipMalloc(&out, 1 << 24);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int blocks : {256, 512, 1024, 2048}) {
    const int iters = 2000;
    hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0, 2.0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = double(blocks) * 4 /*waves*/ * iters * 8 * 16 * 16 * 4 * 2;
    printf("blocks %5d: %.3f ms  %.1f TFLOP/s fp64 MFMA\n", blocks, ms, flop / ms / 1e9);
  }
  return 0;
}
