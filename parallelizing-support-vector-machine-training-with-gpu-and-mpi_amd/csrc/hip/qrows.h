// Kernel values computed from the rows themselves (no stored Gram): the quantised-row layout of the
// exact-integer Gram (igram.hip) or FP64 rows.  Shared by the row-cache solvers (rowcache.hip: the
// graph-replayed select/step pair; smo.hip: the persistent solver with a cached row source).
//
// kval<true> reproduces igram_tri_kernel's arithmetic exactly (int32 group cross terms, the
// group-ordered FP64 flushes, the same dist and exp expressions), so a computed row is
// bit-identical to the resident Gram's and every solver follows the same trajectory.
#pragma once
#include <cstdint>

#include "hip_util.h"

namespace svm355 {

struct QRows {
  const int8_t* Q;       // n x kq centred int8 rows (permuted columns)
  const int32_t* N0;     // exact main-group squared norms
  const double* WN;      // weighted extra-group norms
  const double* step_w;  // per 32-column k-step below main0: group weight at its last step, else 0
  int kq, main_step0;
  double w0;
  // Optional chunk-interleaved copy of Q for per-element row walks (kval2): 16-byte chunk c of row
  // i at Qt + (c * n_rows + i) * 16, so the 64 lanes of a wave reading chunk c of 64 consecutive
  // rows issue one contiguous 1 KB load instead of 64 scattered 16-byte pieces.
  const int8_t* Qt;
  int64_t n_rows;
  // FP64 mode (INT = false)
  const double* X;
  const double* sqn;
  int64_t ld, d;
};

template <bool INT>
__device__ __forceinline__ double kval(const QRows& q, int64_t a, int64_t b, double neg_gamma) {
  if (a == b) return 1.0;
  if constexpr (INT) {
    const int4* pa = reinterpret_cast<const int4*>(q.Q + a * int64_t(q.kq));
    const int4* pb = reinterpret_cast<const int4*>(q.Q + b * int64_t(q.kq));
    const int nsteps = q.kq / 32;
    int32_t acc = 0;
    double x = 0.0;
    for (int s = 0; s < nsteps; ++s) {
      const int4 a0 = pa[2 * s], a1 = pa[2 * s + 1], b0 = pb[2 * s], b1 = pb[2 * s + 1];
      acc = __builtin_amdgcn_sdot4(a0.x, b0.x, acc, false);
      acc = __builtin_amdgcn_sdot4(a0.y, b0.y, acc, false);
      acc = __builtin_amdgcn_sdot4(a0.z, b0.z, acc, false);
      acc = __builtin_amdgcn_sdot4(a0.w, b0.w, acc, false);
      acc = __builtin_amdgcn_sdot4(a1.x, b1.x, acc, false);
      acc = __builtin_amdgcn_sdot4(a1.y, b1.y, acc, false);
      acc = __builtin_amdgcn_sdot4(a1.z, b1.z, acc, false);
      acc = __builtin_amdgcn_sdot4(a1.w, b1.w, acc, false);
      if (s < q.main_step0) {
        const double wg = q.step_w[s];
        if (wg != 0.0) {  // igram_tri_kernel's group flush, same order and expression
          x = __builtin_fma(wg, double(acc), x);
          acc = 0;
        }
      }
    }
    const int32_t D0 = q.N0[a] + q.N0[b] - 2 * acc;
    double dist = q.w0 * double(D0);
    if (q.main_step0 > 0) dist += (q.WN[a] + q.WN[b]) - 2.0 * x;
    dist = dist > 0.0 ? dist : 0.0;
    return exp(neg_gamma * dist);
  } else {
    const double* xa = q.X + a * q.ld;
    const double* xb = q.X + b * q.ld;
    double dot = 0.0;
    for (int64_t k = 0; k < q.d; ++k) dot += xa[k] * xb[k];
    double dist = q.sqn[a] + q.sqn[b] - 2.0 * dot;
    dist = dist > 0.0 ? dist : 0.0;
    return exp(neg_gamma * dist);
  }
}

// K(a, i) and K(b, i) in one pass over row i (a != i, b != i handled like kval): the row-cache
// miss path computes both rows of the pair for its slice while reading each Q row once.
template <bool INT>
__device__ __forceinline__ void kval2(const QRows& q, int64_t a, int64_t b, int64_t i, double neg_gamma,
                                      double* ka, double* kb) {
  if constexpr (INT) {
    const int4* pa = reinterpret_cast<const int4*>(q.Q + a * int64_t(q.kq));
    const int4* pb = reinterpret_cast<const int4*>(q.Q + b * int64_t(q.kq));
    // row i: interleaved chunks (stride n_rows chunks) when available, else the row-major row
    const int4* pi = q.Qt ? reinterpret_cast<const int4*>(q.Qt) + i : reinterpret_cast<const int4*>(q.Q + i * int64_t(q.kq));
    const int64_t cs = q.Qt ? q.n_rows : 1;
    const int nsteps = q.kq / 32;
    int32_t acca = 0, accb = 0;
    double xa = 0.0, xb = 0.0;
#pragma unroll 4
    for (int s = 0; s < nsteps; ++s) {
      const int4 i0 = pi[(2 * s) * cs], i1 = pi[(2 * s + 1) * cs];
      const int4 a0 = pa[2 * s], a1 = pa[2 * s + 1], b0 = pb[2 * s], b1 = pb[2 * s + 1];
      acca = __builtin_amdgcn_sdot4(a0.x, i0.x, acca, false);
      acca = __builtin_amdgcn_sdot4(a0.y, i0.y, acca, false);
      acca = __builtin_amdgcn_sdot4(a0.z, i0.z, acca, false);
      acca = __builtin_amdgcn_sdot4(a0.w, i0.w, acca, false);
      acca = __builtin_amdgcn_sdot4(a1.x, i1.x, acca, false);
      acca = __builtin_amdgcn_sdot4(a1.y, i1.y, acca, false);
      acca = __builtin_amdgcn_sdot4(a1.z, i1.z, acca, false);
      acca = __builtin_amdgcn_sdot4(a1.w, i1.w, acca, false);
      accb = __builtin_amdgcn_sdot4(b0.x, i0.x, accb, false);
      accb = __builtin_amdgcn_sdot4(b0.y, i0.y, accb, false);
      accb = __builtin_amdgcn_sdot4(b0.z, i0.z, accb, false);
      accb = __builtin_amdgcn_sdot4(b0.w, i0.w, accb, false);
      accb = __builtin_amdgcn_sdot4(b1.x, i1.x, accb, false);
      accb = __builtin_amdgcn_sdot4(b1.y, i1.y, accb, false);
      accb = __builtin_amdgcn_sdot4(b1.z, i1.z, accb, false);
      accb = __builtin_amdgcn_sdot4(b1.w, i1.w, accb, false);
      if (s < q.main_step0) {
        const double wg = q.step_w[s];
        if (wg != 0.0) {
          xa = __builtin_fma(wg, double(acca), xa);
          xb = __builtin_fma(wg, double(accb), xb);
          acca = 0;
          accb = 0;
        }
      }
    }
    double da = q.w0 * double(q.N0[a] + q.N0[i] - 2 * acca);
    double db = q.w0 * double(q.N0[b] + q.N0[i] - 2 * accb);
    if (q.main_step0 > 0) {
      da += (q.WN[a] + q.WN[i]) - 2.0 * xa;
      db += (q.WN[b] + q.WN[i]) - 2.0 * xb;
    }
    da = da > 0.0 ? da : 0.0;
    db = db > 0.0 ? db : 0.0;
    *ka = a == i ? 1.0 : exp(neg_gamma * da);
    *kb = b == i ? 1.0 : exp(neg_gamma * db);
  } else {
    *ka = kval<false>(q, a, i, neg_gamma);
    *kb = kval<false>(q, b, i, neg_gamma);
  }
}

}  // namespace svm355
