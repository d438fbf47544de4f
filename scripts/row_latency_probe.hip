// Latency of one K(W, W) row load as the inner solve issues it (256 threads x two 16-byte loads = one
// 8 KB row), measured in clock64 ticks per dependent row load by one workgroup:
//   * rows written just before by a many-workgroup kernel on every XCD (first touch from this CU),
//   * the same rows again (now in this XCD's L2: a repeat within an outer iteration),
//   * a cycle of 64 rows (512 KB, L2-resident, beyond the 32 KB vector L1),
//   * rows after a 512 MB streaming pass (HBM),
//   * 256 rows (2 MB) written or read beforehand only by the workgroups on the probe's XCD (is a line
//     another kernel left in this XCD's L2 still there for the next kernel?).
// Design input for the inner-solve floor (profiles/r4_decomp_inner_floor.txt).
//   hipcc --offload-arch=gfx950 -O3 -o scripts/row_latency_probe scripts/row_latency_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr int kRows = 1024, kLd = 1024, kNT = 256;

__global__ void fill_kernel(double* K, double s) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < int64_t(kRows) * kLd) K[i] = s + double(i % 977) * 1e-9;
}

__device__ inline int xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15; }

// only the workgroups on XCD `x` work (rows [0, 256)): the lines pass through that XCD's L2
__global__ void fill_xcd_kernel(double* K, double s, int x, int nwg_x) {
  if (xcc_id() != x) return;
  const int k = blockIdx.x / 8;  // this XCD's k-th workgroup (round-robin dispatch)
  for (int64_t i = int64_t(k) * blockDim.x + threadIdx.x; i < 256ll * kLd; i += int64_t(nwg_x) * blockDim.x)
    K[i] = s + double(i % 977) * 1e-9;
}

__global__ void touch_xcd_kernel(const double* K, int x, int nwg_x, double* sink) {
  if (xcc_id() != x) return;
  const int k = blockIdx.x / 8;
  double acc = 0.0;
  for (int64_t i = int64_t(k) * blockDim.x + threadIdx.x; i < 256ll * kLd; i += int64_t(nwg_x) * blockDim.x)
    acc += K[i];
  if (acc == 1234.5) sink[0] = acc;
}

__global__ void stream_kernel(const double4* src, int64_t n, double* sink) {
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    acc += src[i].x + src[i].w;
  if (acc == 1234.5) sink[0] = acc;
}

// one workgroup: nseq dependent row loads (the next row depends on the loaded values through a zero)
__global__ void __launch_bounds__(kNT) probe_kernel(const double* K, const int* seq, int nseq, long long* ticks,
                                                    double* sink, int* xcc) {
  __shared__ double red[kNT / 64];
  const int t = threadIdx.x;
  double acc = 0.0;
  int dep = 0;
  const long long t0 = clock64();
  for (int s = 0; s < nseq; ++s) {
    const int r = seq[s] + dep;
    const double2* src = reinterpret_cast<const double2*>(K + int64_t(r) * kLd) + t;
    const double2 a = src[0], b = src[kNT];
    const double v = a.x + a.y + b.x + b.y;
    acc += v;
    dep = int(v * 0.0);  // a data dependence: the next row waits for this one
  }
  const long long t1 = clock64();
  double w = acc;
  for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o);
  if ((t & 63) == 0) red[t >> 6] = w;
  __syncthreads();
  if (t == 0) {
    ticks[0] = t1 - t0;
    xcc[0] = xcc_id();
    sink[0] = red[0] + red[1] + red[2] + red[3];
  }
}

int main() {
  double *K, *sink, *big;
  int *dseq, *dxcc;
  long long* dt;
  const int64_t nbig = (512ll << 20) / 32;
  CK(hipMalloc(&K, sizeof(double) * kRows * kLd));
  CK(hipMalloc(&big, 32 * nbig));
  CK(hipMemset(big, 0, 32 * nbig));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&dt, 64));
  CK(hipMalloc(&dseq, sizeof(int) * 4096));
  CK(hipMalloc(&dxcc, 64));
  std::vector<int> uniq(kRows), cyc(1024), u256(256), twice(512);
  srand(7);
  for (int i = 0; i < kRows; ++i) uniq[i] = i;
  for (int i = kRows - 1; i > 0; --i) std::swap(uniq[i], uniq[rand() % (i + 1)]);
  for (int i = 0; i < 1024; ++i) cyc[i] = uniq[i % 64];
  for (int i = 0; i < 256; ++i) u256[i] = i;
  for (int i = 255; i > 0; --i) std::swap(u256[i], u256[rand() % (i + 1)]);
  for (int i = 0; i < 512; ++i) twice[i] = u256[i % 256];
  int px = 0;
  // mode: 0 nothing, 1 refill everywhere, 2 flush, 3 refill rows < 256 from the probe's XCD only,
  // 4 refill everywhere then read rows < 256 from the probe's XCD only
  auto run = [&](const std::vector<int>& seq, const char* what, int mode) {
    CK(hipMemcpy(dseq, seq.data(), sizeof(int) * seq.size(), hipMemcpyHostToDevice));
    if (mode == 1 || mode == 4) fill_kernel<<<(kRows * kLd + 255) / 256, 256>>>(K, 1.0);
    if (mode == 2) stream_kernel<<<4096, 256>>>(reinterpret_cast<const double4*>(big), nbig, sink);
    if (mode == 3) fill_xcd_kernel<<<8 * 32, 256>>>(K, 2.0, px, 32);
    if (mode == 4) touch_xcd_kernel<<<8 * 32, 256>>>(K, px, 32, sink);
    probe_kernel<<<1, kNT>>>(K, dseq, int(seq.size()), dt, sink, dxcc);
    CK(hipGetLastError());
    long long h = 0;
    CK(hipMemcpy(&h, dt, sizeof(h), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&px, dxcc, sizeof(int), hipMemcpyDeviceToHost));
    printf("%-62s %7.1f ticks per row load (%zu loads, probe on XCD %d)\n", what, double(h) / seq.size(),
           seq.size(), px);
  };
  for (int rep = 0; rep < 2; ++rep) {
    run(uniq, "unique rows, just written on every XCD", 1);
    run(uniq, "the same rows again (8 MB: more than the L2)", 0);
    run(cyc, "cycle of 64 rows (512 KB)", 0);
    run(uniq, "unique rows after a 512 MB streaming pass (HBM)", 2);
    run(u256, "256 unique rows, just written on every XCD", 1);
    run(twice, "256 rows twice in one kernel, just written on every XCD", 1);
    run(u256, "256 unique rows, the previous kernel read them (same XCD)", 0);
    run(u256, "256 unique rows, just written from the probe's XCD only", 3);
    run(u256, "256 unique rows, written everywhere, then read on the XCD", 4);
  }
  CK(hipDeviceSynchronize());
  CK(hipFree(K));
  CK(hipFree(big));
  CK(hipFree(sink));
  CK(hipFree(dt));
  CK(hipFree(dseq));
  CK(hipFree(dxcc));
  return 0;
}
