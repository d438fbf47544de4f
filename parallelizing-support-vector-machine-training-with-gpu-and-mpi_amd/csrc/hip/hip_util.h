// Shared HIP/CDNA4 helpers for the svm355 device library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "svm355.h"

namespace svm355 {
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
}

#define SVMD_CHECK(expr)                                                                     \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) {                                                                  \
      svm355::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,                 \
                        hipGetErrorString(_e));                                              \
      return SVM_ERR_DEVICE;                                                                 \
    }                                                                                        \
  } while (0)

#define SVMD_LAUNCH_CHECK() SVMD_CHECK(hipGetLastError())

// One trivial kernel per translation unit.  Every .hip file is its own fat binary, and HIP loads a
// code object at the first launch of any kernel in it: 0.5-9.3 ms per file on MI355X (smo.hip's is the
// largest), which the first fit paid inside its timed region (profiles/r5_cold_fit_trace.txt).
// svmd_create launches every file's kernel (tu_warm_all, capi.hip), so no fit loads a code object.
#define SVMD_TU_WARM(name)                                                                  \
  namespace svm355 {                                                                        \
  namespace {                                                                               \
  __global__ void tu_warm_kernel_##name(int* p) {                                           \
    if (p && threadIdx.x == 0) *p = 0;                                                      \
  }                                                                                         \
  }                                                                                         \
  int tu_warm_##name(hipStream_t s) {                                                       \
    hipLaunchKernelGGL(tu_warm_kernel_##name, dim3(1), dim3(64), 0, s, nullptr);            \
    return hipPeekAtLastError() == hipSuccess ? 0 : 1;                                      \
  }                                                                                         \
  }

namespace svm355 {

constexpr int kWave = 64;  // CDNA wavefront width (hard-coded per the gfx950 guide)

// Rows of device feature matrices are padded to a multiple of kKPad doubles (zero-filled) so the
// MFMA Gram kernel needs no k-tail handling and every row start is 16-byte aligned.
constexpr int64_t kKPad = 16;
inline int64_t padded_dim(int64_t d) { return (d + kKPad - 1) / kKPad * kKPad; }

// (value, index) pair with the serial lowest-index tie-break: `b` replaces `a` when it is
// strictly better, or equal with a smaller index.  Sentinels carry index = INT64_MAX.
struct ArgPair {
  double v;
  int64_t i;
};

__device__ __forceinline__ bool better_min(double av, int64_t ai, double bv, int64_t bi) {
  return bv < av || (bv == av && bi < ai);
}
__device__ __forceinline__ bool better_max(double av, int64_t ai, double bv, int64_t bi) {
  return bv > av || (bv == av && bi < ai);
}

// Full-wave (64-lane) argmin/argmax butterfly; every lane ends with the wave result.
__device__ __forceinline__ void wave_argmin(double& v, int64_t& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(v, off, kWave);
    const int64_t oi = __shfl_xor(i, off, kWave);
    if (better_min(v, i, ov, oi)) {
      v = ov;
      i = oi;
    }
  }
}
__device__ __forceinline__ void wave_argmax(double& v, int64_t& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(v, off, kWave);
    const int64_t oi = __shfl_xor(i, off, kWave);
    if (better_max(v, i, ov, oi)) {
      v = ov;
      i = oi;
    }
  }
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

}  // namespace svm355
