// L1 preprocessing kernels (gfx950): column min/max, min-max scaling fused with the squared row
// norms the MFMA RBF path needs, and row gathers.
//
// Reference: find_min_max (gpu_svm_main3.cu:62-95) runs a multi-pass 32x32 tree reduction that
// needs four n x d FP64 scratch copies (~1.5 GB at 60k, :540-548); scale_features (:100-116) is a
// separate elementwise pass with a 32-bit index.  Here: one streaming pass over X for min/max with
// per-block column partials (no n x d scratch), then one pass that scales in place and emits
// ||x||^2 (one wave per row, fixed butterfly order -> deterministic), 64-bit indexing throughout.
#include "ctx.h"

namespace svm355 {
namespace {

constexpr int kColsPerBlock = 64;  // one column per lane of a wave
constexpr int kRowLanes = 4;       // 4 waves stride the rows

__global__ __launch_bounds__(256) void minmax_partial_kernel(const double* __restrict__ X, int64_t n,
                                                             int64_t d, int64_t ld,
                                                             double* __restrict__ pmin,
                                                             double* __restrict__ pmax) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c = int64_t(blockIdx.x) * kColsPerBlock + lane;
  const int64_t rstride = int64_t(gridDim.y) * kRowLanes;
  double lo = __builtin_inf(), hi = -__builtin_inf();
  bool nan = false;  // fmin / fmax drop NaN: a NaN anywhere in the column makes both of its bounds NaN
  if (c < d) {
    for (int64_t r = int64_t(blockIdx.y) * kRowLanes + wv; r < n; r += rstride) {
      const double v = X[r * ld + c];
      lo = fmin(lo, v);
      hi = fmax(hi, v);
      nan |= v != v;
    }
  }
  if (nan) lo = hi = __builtin_nan("");
  __shared__ double smin[kRowLanes][kColsPerBlock], smax[kRowLanes][kColsPerBlock];
  smin[wv][lane] = lo;
  smax[wv][lane] = hi;
  __syncthreads();
  if (wv == 0 && c < d) {
#pragma unroll
    for (int w = 1; w < kRowLanes; ++w) {
      nan |= smin[w][lane] != smin[w][lane] || lo != lo;
      lo = fmin(lo, smin[w][lane]);
      hi = fmax(hi, smax[w][lane]);
    }
    if (nan) lo = hi = __builtin_nan("");
    pmin[int64_t(blockIdx.y) * d + c] = lo;
    pmax[int64_t(blockIdx.y) * d + c] = hi;
  }
}

__global__ __launch_bounds__(256) void minmax_final_kernel(const double* __restrict__ pmin,
                                                           const double* __restrict__ pmax, int parts,
                                                           int64_t d, double* __restrict__ mn,
                                                           double* __restrict__ mx) {
  const int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= d) return;
  double lo = pmin[c], hi = pmax[c];
  bool nan = lo != lo;  // a NaN partial (a NaN in the column) stays NaN: fmin / fmax would drop it
  // 8 partials' loads in flight ahead of the in-order folds (same order, same result)
  int p = 1;
  for (; p + 8 <= parts; p += 8) {
    double a[8], z[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a[u] = pmin[int64_t(p + u) * d + c];
      z[u] = pmax[int64_t(p + u) * d + c];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      nan |= a[u] != a[u];
      lo = fmin(lo, a[u]);
      hi = fmax(hi, z[u]);
    }
  }
  for (; p < parts; ++p) {
    const double a = pmin[int64_t(p) * d + c];
    nan |= a != a;
    lo = fmin(lo, a);
    hi = fmax(hi, pmax[int64_t(p) * d + c]);
  }
  mn[c] = nan ? __builtin_nan("") : lo;
  mx[c] = nan ? __builtin_nan("") : hi;
}

// One wave per row.  mn == nullptr -> norms only.
__global__ __launch_bounds__(256) void scale_norm_kernel(double* __restrict__ X, int64_t n, int64_t d,
                                                         int64_t ld, const double* __restrict__ mn,
                                                         const double* __restrict__ mx,
                                                         double* __restrict__ sqn) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= n) return;
  double* xr = X + row * ld;
  double acc = 0.0;
  for (int64_t c = lane; c < d; c += 64) {
    double v = xr[c];
    if (mn) {
      double range = mx[c] - mn[c];
      if (range < 1e-12) range = 1.0;
      v = (v - mn[c]) / range;  // true division, bit-identical to the CPU reference
      xr[c] = v;
    }
    acc += v * v;
  }
  acc = wave_sum(acc);
  if (lane == 0 && sqn) sqn[row] = acc;
}

__global__ __launch_bounds__(256) void gather_rows_kernel(const double* __restrict__ src, int64_t ld,
                                                          const int64_t* __restrict__ idx, int64_t k,
                                                          double* __restrict__ dst) {
  for (int64_t r = blockIdx.x; r < k; r += gridDim.x) {
    const double2* s = reinterpret_cast<const double2*>(src + idx[r] * ld);
    double2* o = reinterpret_cast<double2*>(dst + r * ld);
    for (int64_t c = threadIdx.x; c < ld / 2; c += blockDim.x) o[c] = s[c];
  }
}

// Compact uint8 pixel rows (n x d, contiguous) -> zero-padded FP64 rows (n x ld).  Pixel data are
// uploaded as bytes (8x less PCIe traffic) and widened on the device; every value is exact in FP64.
__global__ __launch_bounds__(256) void widen_u8_kernel(const uint8_t* __restrict__ src, int64_t n, int64_t d,
                                                       int64_t ld, double* __restrict__ dst) {
  const int64_t total = n * ld;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = i / ld, c = i - r * ld;
    dst[i] = c < d ? double(src[r * d + c]) : 0.0;
  }
}

// minmax_partial_kernel on uint8 pixel rows (n x d contiguous): min / max of the widened values are
// the widened min / max, so the statistics equal those of the FP64 rows exactly.
__global__ __launch_bounds__(256) void minmax_u8_partial_kernel(const uint8_t* __restrict__ X, int64_t n, int64_t d,
                                                                double* __restrict__ pmin, double* __restrict__ pmax) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c = int64_t(blockIdx.x) * kColsPerBlock + lane;
  const int64_t rstride = int64_t(gridDim.y) * kRowLanes;
  int lo = 255, hi = 0;
  bool any = false;
  if (c < d) {
    for (int64_t r = int64_t(blockIdx.y) * kRowLanes + wv; r < n; r += rstride) {
      const int v = X[r * d + c];
      lo = min(lo, v);
      hi = max(hi, v);
      any = true;
    }
  }
  __shared__ int smin[kRowLanes][kColsPerBlock], smax[kRowLanes][kColsPerBlock];
  __shared__ bool sany[kRowLanes][kColsPerBlock];
  smin[wv][lane] = lo;
  smax[wv][lane] = hi;
  sany[wv][lane] = any;
  __syncthreads();
  if (wv == 0 && c < d) {
#pragma unroll
    for (int w = 1; w < kRowLanes; ++w) {
      lo = min(lo, smin[w][lane]);
      hi = max(hi, smax[w][lane]);
      any = any || sany[w][lane];
    }
    pmin[int64_t(blockIdx.y) * d + c] = any ? double(lo) : __builtin_inf();
    pmax[int64_t(blockIdx.y) * d + c] = any ? double(hi) : -__builtin_inf();
  }
}

// Scaled FP64 rows idx[0..k) of uint8 pixel rows, zero padded to ld, and their squared norms: the
// widen + scale_norm arithmetic per row (same per-lane column order, same wave_sum), so the rows and
// norms equal those of the scaled FP64 matrix bit for bit.  One wave per output row.
__global__ __launch_bounds__(256) void sv_rows_u8_kernel(const uint8_t* __restrict__ X, int64_t d,
                                                         const int64_t* __restrict__ idx, int64_t k,
                                                         const double* __restrict__ mn, const double* __restrict__ mx,
                                                         double* __restrict__ out, int64_t ld, double* __restrict__ sqn) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= k) return;
  const uint8_t* xr = X + idx[row] * d;
  double* o = out + row * ld;
  double acc = 0.0;
  for (int64_t c = lane; c < d; c += 64) {
    double range = mx[c] - mn[c];
    if (range < 1e-12) range = 1.0;
    const double v = (double(xr[c]) - mn[c]) / range;
    o[c] = v;
    acc += v * v;
  }
  for (int64_t c = d + lane; c < ld; c += 64) o[c] = 0.0;
  acc = wave_sum(acc);
  if (lane == 0) sqn[row] = acc;
}

}  // namespace

int launch_minmax_u8(hipStream_t s, const uint8_t* X, int64_t n, int64_t d, double* mn, double* mx, double* scratch,
                     size_t scratch_doubles) {
  const int gx = int((d + kColsPerBlock - 1) / kColsPerBlock);
  int parts = int(std::min<int64_t>((n + kRowLanes - 1) / kRowLanes, std::max(1, 2048 / gx)));
  parts = int(std::min<int64_t>(parts, int64_t(scratch_doubles / size_t(2 * d))));
  if (parts < 1) {
    set_error("launch_minmax_u8: scratch too small");
    return SVM_ERR_INTERNAL;
  }
  double* pmin = scratch;
  double* pmax = scratch + size_t(parts) * size_t(d);
  hipLaunchKernelGGL(minmax_u8_partial_kernel, dim3(gx, parts), dim3(256), 0, s, X, n, d, pmin, pmax);
  SVMD_LAUNCH_CHECK();
  hipLaunchKernelGGL(minmax_final_kernel, dim3(int((d + 255) / 256)), dim3(256), 0, s, pmin, pmax, parts, d, mn, mx);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

int launch_sv_rows_u8(hipStream_t s, const uint8_t* X, int64_t d, const int64_t* idx, int64_t k, const double* mn,
                      const double* mx, double* out, int64_t ld, double* sqn) {
  if (k <= 0) return SVM_OK;
  hipLaunchKernelGGL(sv_rows_u8_kernel, dim3(unsigned((k + 3) / 4)), dim3(256), 0, s, X, d, idx, k, mn, mx, out, ld,
                     sqn);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

int launch_widen_u8(hipStream_t s, const uint8_t* src, int64_t n, int64_t d, int64_t ld, double* dst) {
  if (n <= 0) return SVM_OK;
  const int64_t blocks = std::min<int64_t>((n * ld + 255) / 256, 256 * 64);
  hipLaunchKernelGGL(widen_u8_kernel, dim3(unsigned(blocks)), dim3(256), 0, s, src, n, d, ld, dst);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

int launch_minmax(hipStream_t s, const double* X, int64_t n, int64_t d, int64_t ld, double* mn,
                  double* mx, double* scratch, size_t scratch_doubles) {
  const int gx = int((d + kColsPerBlock - 1) / kColsPerBlock);
  // ~2k blocks fill the 256 CUs; each partial row is d doubles (x2 for min and max).
  int parts = int(std::min<int64_t>((n + kRowLanes - 1) / kRowLanes, std::max(1, 2048 / gx)));
  parts = int(std::min<int64_t>(parts, int64_t(scratch_doubles / size_t(2 * d))));
  if (parts < 1) {
    set_error("launch_minmax: scratch too small");
    return SVM_ERR_INTERNAL;
  }
  double* pmin = scratch;
  double* pmax = scratch + size_t(parts) * size_t(d);
  hipLaunchKernelGGL(minmax_partial_kernel, dim3(gx, parts), dim3(256), 0, s, X, n, d, ld, pmin, pmax);
  SVMD_LAUNCH_CHECK();
  hipLaunchKernelGGL(minmax_final_kernel, dim3(int((d + 255) / 256)), dim3(256), 0, s, pmin, pmax, parts,
                     d, mn, mx);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

int launch_scale_norms(hipStream_t s, double* X, int64_t n, int64_t d, int64_t ld, const double* mn,
                       const double* mx, double* sqn) {
  if (n <= 0) return SVM_OK;
  const int64_t blocks = (n + 3) / 4;
  hipLaunchKernelGGL(scale_norm_kernel, dim3(unsigned(blocks)), dim3(256), 0, s, X, n, d, ld, mn, mx, sqn);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

int launch_gather_rows(hipStream_t s, const double* src, int64_t ld, const int64_t* idx, int64_t k,
                       double* dst) {
  if (k <= 0) return SVM_OK;
  if (ld % 2) {
    set_error("gather_rows: ld must be even");
    return SVM_ERR_ARG;
  }
  const unsigned grid = unsigned(std::min<int64_t>(k, 1 << 20));
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid), dim3(256), 0, s, src, ld, idx, k, dst);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

}  // namespace svm355

SVMD_TU_WARM(prep_kernels)
