// Probe: the summation order / rounding of v_mfma_f64_16x16x4f64 within one instruction, to decide whether
// a left-looking Cholesky's row updates (ascending fma chains) may run on MFMA bit-identically to the CPU
// oracle.  For T random trials: lane l supplies A[l & 15][l >> 4], B[l >> 4][l & 15], and C; D is written
// with its layout (col = lane & 15, row = (lane >> 4) + 4 r).  The host compares every D entry with
//   seq: c = fma(a0, b0, c); c = fma(a1, b1, c); c = fma(a2, b2, c); c = fma(a3, b3, c)   (k = 0..3)
//   rev: the same chain for k = 3..0
// and prints the number of entries matching each (bit for bit).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const double* A, const double* B, const double* Cin, double* D, int trials) {
  const int lane = threadIdx.x;
  for (int tr = 0; tr < trials; ++tr) {
    const double* a = A + tr * 64;
    const double* b = B + tr * 64;
    const double* c = Cin + tr * 256;
    const int col = lane & 15, g = lane >> 4;
    f64x4 acc;
    for (int r = 0; r < 4; ++r) acc[r] = c[(g + 4 * r) * 16 + col];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[(lane & 15) * 4 + (lane >> 4)], b[(lane >> 4) * 16 + (lane & 15)], acc,
                                               0, 0, 0);
    for (int r = 0; r < 4; ++r) D[tr * 256 + (g + 4 * r) * 16 + col] = acc[r];
  }
}

int main() {
  const int T = 2000;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  std::vector<double> A(T * 64), B(T * 64), C(T * 256), D(T * 256);
  for (int t = 0; t < T; ++t) {
    const double sa = std::ldexp(1.0, int(rng() % 40) - 20), sc = std::ldexp(1.0, int(rng() % 40) - 20);
    for (int i = 0; i < 64; ++i) {  // A[row][k] at row * 4 + k
      A[t * 64 + i] = u(rng) * sa * ((rng() & 7) == 0 ? 1e8 : 1.0);
      B[t * 64 + i] = u(rng);
    }
    for (int i = 0; i < 256; ++i) C[t * 256 + i] = u(rng) * sc;
  }
  double *dA, *dB, *dC, *dD;
  hipMalloc(&dA, A.size() * 8);
  hipMalloc(&dB, B.size() * 8);
  hipMalloc(&dC, C.size() * 8);
  hipMalloc(&dD, D.size() * 8);
  hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, T);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  hipMemcpy(D.data(), dD, D.size() * 8, hipMemcpyDeviceToHost);
  long seq = 0, rev = 0, tot = 0;
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        const double* a = &A[t * 64 + i * 4];
        double s = C[t * 256 + i * 16 + j], r = s;
        for (int k = 0; k < 4; ++k) s = std::fma(a[k], B[t * 64 + k * 16 + j], s);
        for (int k = 3; k >= 0; --k) r = std::fma(a[k], B[t * 64 + k * 16 + j], r);
        const double d = D[t * 256 + i * 16 + j];
        seq += d == s;
        rev += d == r;
        ++tot;
      }
  printf("entries %ld: seq-fma match %ld, reverse-fma match %ld\n", tot, seq, rev);
  return 0;
}
