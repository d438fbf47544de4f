// L2 kernel evaluation, exact-integer path: RBF Gram of integer-valued features on int8 MFMA.
//
// MNIST-shaped inputs are integer pixel intensities, and after the reference's min-max scaling
// (main3.cpp:74-89) feature j of every row is x_j = q_j / r_j with q_j = p_j - min_j an integer in
// [0, r_j] and r_j = max_j - min_j.  So
//
//     ||x_a - x_b||^2 = sum_j w_j (q_aj - q_bj)^2,           w_j = 1 / r_j^2
//                     = w0 * D_ab + sum_{j in corr} (w_j - w0) (q_aj - q_bj)^2
//
// where w0 is the weight shared by most columns (r_j = 255 on MNIST) and
// D_ab = sum_j (q_aj - q_bj)^2 = N_a + N_b - 2 * I_ab is an EXACT integer: I_ab = sum_j q'_aj q'_bj
// on biased int8 operands q' = q - 128 (the bias cancels in the difference) is one
// v_mfma_i32_32x32x32_i8 GEMM with int32 accumulation.  The few columns whose range differs
// ("correction" columns, <= 12% on MNIST-shaped data) are placed first in a permuted column order
// and their weighted term is an FP64 v_mfma_f64_16x16x4_f64 GEMM fed from the SAME staged int8
// tiles (converted in registers and scaled by sqrt|delta_j|, delta_j = w_j - w0).  The distance is therefore
// computed without the catastrophic ||a||^2 + ||b||^2 - 2ab cancellation of the plain FP64 path
// (gram_mfma.hip): the integer part is exact and the FP64 part is small, so every kernel value is
// FP64-accurate (tests/test_gpu_kernels.py checks |K - K_exact| <= 1e-15).
//
// Reference: calc_kernel_matrix (gpu_svm_main3.cu:137-147) evaluates one FP64 row per launch with
// a d-long scalar loop per thread.  Here the whole upper-triangular Gram is produced in one launch
// (128x128 tiles, 4 waves of 64x64, XCD-aware tile order), the mirror half is written through an
// LDS transpose, and the FP64 MFMA work is ~8x smaller than the plain FP64 Gram.
#include <algorithm>
#include <cmath>
#include <map>
#include <vector>

#include "ctx.h"
#include "tile_map.h"

namespace svm355 {
namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int QBM = 128;        // tile rows / cols
constexpr int QBK = 64;         // int8 columns per LDS stage
constexpr int QLS = QBK + 16;   // LDS row stride in bytes (80: conflict-free ds_read_b128 rows)
constexpr int kMaxCorr = 1024;  // correction columns kept in LDS (scales, centres)
constexpr int kStageBytes = 2 * QBM * QLS + kMaxCorr * 24;
constexpr int kEpiBytes = 4 * 32 * 33 * 4 + 4 * 16 * 17 * 8;  // int transpose + mirror scratch
constexpr int kSmemBytes = kStageBytes > kEpiBytes ? kStageBytes : kEpiBytes;

// ---- quantisation: one wave per row.  Writes the permuted biased int8 row, N = sum q'^2 (exact)
// and cN = sum_{k < kc} delta_k (q_k - c_k)^2 (correction operand centred on c_k = floor(r_k / 2),
// which keeps the FP64 correction terms small); flags any value that is not an integer in [0, 255].
__global__ __launch_bounds__(256) void quantize_rows_kernel(
    const double* __restrict__ X, int64_t n, int64_t ld, const int32_t* __restrict__ perm,
    const double* __restrict__ rmul, const double* __restrict__ delta, const double* __restrict__ cen, int kc,
    int kq, int8_t* __restrict__ Q, int32_t* __restrict__ Nq, double* __restrict__ cN, unsigned* __restrict__ fail) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const double* xr = X + row * ld;
  int32_t* qr = reinterpret_cast<int32_t*>(Q + row * int64_t(kq));
  int32_t nacc = 0;
  double cacc = 0.0;
  bool bad = false;
  for (int w = lane; w < kq / 4; w += 64) {
    uint32_t word = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int k = 4 * w + b;
      const int j = perm[k];
      int qq = 0;
      if (j >= 0) {
        const double v = xr[j] * rmul[k];
        const double q = rint(v);
        bad |= !(fabs(v - q) <= 1e-6) || q < 0.0 || q > 255.0;
        qq = int(q) - 128;
        nacc += qq * qq;
        if (k < kc) {
          const double qc = q - cen[k];  // centred correction operand (exact)
          cacc += delta[k] * (qc * qc);
        }
      }
      word |= uint32_t(uint8_t(int8_t(qq))) << (8 * b);
    }
    qr[w] = int32_t(word);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) nacc += __shfl_xor(nacc, off, kWave);
  cacc = wave_sum(cacc);
  if (lane == 0) {
    Nq[row] = nacc;
    cN[row] = cacc;
  }
  if (__any(bad) && lane == 0) atomicOr(fail, 1u);
}

__device__ __forceinline__ double sbyte(uint32_t w, int s) {  // signed byte s of w -> double
  return double(int32_t(w << (24 - 8 * s)) >> 24);
}

// Upper-triangular tiles of K = exp(-gamma * dist) for the n quantised rows, each off-diagonal
// tile also stored transposed.  kc = correction columns (multiple of 16, <= kMaxCorr), kq = total
// int8 columns (multiple of QBK).
template <bool CORR>
__global__ __launch_bounds__(256, 2) void igram_tri_kernel(
    const int8_t* __restrict__ Q, int64_t n, int kq, int kc, const int32_t* __restrict__ Nq,
    const double* __restrict__ cN, const double* __restrict__ delta, const double* __restrict__ cen, double w0,
    double neg_gamma,
    double* __restrict__ K, int64_t ldk, int64_t tiles) {
  __shared__ __attribute__((aligned(16))) char smem[kSmemBytes];
  char* As = smem;
  char* Bs = smem + QBM * QLS;
  double* dsa = reinterpret_cast<double*>(smem + 2 * QBM * QLS);  // sqrt|delta_k|
  double* dsb = dsa + kMaxCorr;                                     // sign(delta_k) sqrt|delta_k|
  double* dco = dsb + kMaxCorr;                                     // 128 - c_k (byte -> centred q)

  int64_t tm, tn;
  tri_tile(xcd_remap(blockIdx.x, tiles * (tiles + 1) / 2), tiles, tm, tn);
  const int64_t bm = tm * QBM, bn = tn * QBM;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;

  // Both operands carry sqrt|delta| (B also the sign), so the (i, j) and (j, i) products of a
  // diagonal tile are the same two rounded factors: the Gram comes out exactly symmetric.
  if (CORR)
    for (int k = t; k < kc; k += 256) {
      const double sd = sqrt(fabs(delta[k]));
      dsa[k] = sd;
      dsb[k] = delta[k] < 0.0 ? -sd : sd;
      dco[k] = 128.0 - cen[k];
    }

  // Staging: 128 rows x 64 B per operand = 512 x 16 B; thread t copies rows t>>2 and 64 + (t>>2),
  // 16-byte column chunk t&3.
  const int srow = t >> 2, scol = (t & 3) * 16;
  const int64_t ra0 = bm + srow, ra1 = bm + srow + 64, rb0 = bn + srow, rb1 = bn + srow + 64;
  const i32x4 zero4 = {0, 0, 0, 0};
  i32x4 ga[2], gb[2];
  auto gload = [&](int k0) {
    ga[0] = ra0 < n ? *reinterpret_cast<const i32x4*>(Q + ra0 * kq + k0 + scol) : zero4;
    ga[1] = ra1 < n ? *reinterpret_cast<const i32x4*>(Q + ra1 * kq + k0 + scol) : zero4;
    gb[0] = rb0 < n ? *reinterpret_cast<const i32x4*>(Q + rb0 * kq + k0 + scol) : zero4;
    gb[1] = rb1 < n ? *reinterpret_cast<const i32x4*>(Q + rb1 * kq + k0 + scol) : zero4;
  };
  gload(0);

  i32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;
  f64x4 cacc[4][4];
  if (CORR) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) cacc[i][j] = f64x4{0.0, 0.0, 0.0, 0.0};
  }

  const int l32 = lane & 31, h = lane >> 5;
  const int lr = lane & 15, lg = lane >> 4;
  for (int k0 = 0; k0 < kq; k0 += QBK) {
    __syncthreads();
    *reinterpret_cast<i32x4*>(As + srow * QLS + scol) = ga[0];
    *reinterpret_cast<i32x4*>(As + (srow + 64) * QLS + scol) = ga[1];
    *reinterpret_cast<i32x4*>(Bs + srow * QLS + scol) = gb[0];
    *reinterpret_cast<i32x4*>(Bs + (srow + 64) * QLS + scol) = gb[1];
    __syncthreads();
    if (k0 + QBK < kq) gload(k0 + QBK);

    // int8 part: two 32-deep k-steps.  A and B fragments use the same (lane, byte) -> k map, so
    // the product is independent of the hardware's k order inside a step.
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      i32x4 a[2], b[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
        a[mi] = *reinterpret_cast<const i32x4*>(As + (wr * 64 + mi * 32 + l32) * QLS + ks * 32 + 16 * h);
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
        b[nj] = *reinterpret_cast<const i32x4*>(Bs + (wc * 64 + nj * 32 + l32) * QLS + ks * 32 + 16 * h);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj)
          acc[mi][nj] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[mi], b[nj], acc[mi][nj], 0, 0, 0);
    }

    // FP64 correction columns: 16-column chunks of this stage below kc.  Lane group lg at
    // sub-step s uses column 4*lg + s of the chunk (same map for A and B).
    if (CORR) {
#pragma unroll
      for (int c = 0; c < QBK / 16; ++c) {
        const int kb = k0 + 16 * c;
        if (kb >= kc) break;
        uint32_t aw[4], bw[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          aw[mi] = *reinterpret_cast<const uint32_t*>(As + (wr * 64 + mi * 16 + lr) * QLS + 16 * c + 4 * lg);
#pragma unroll
        for (int nj = 0; nj < 4; ++nj)
          bw[nj] = *reinterpret_cast<const uint32_t*>(Bs + (wc * 64 + nj * 16 + lr) * QLS + 16 * c + 4 * lg);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kk = kb + 4 * lg + s;
          const double sa = dsa[kk], sb = dsb[kk], co = dco[kk];
          double af[4], bf[4];
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) af[mi] = (sbyte(aw[mi], s) + co) * sa;
#pragma unroll
          for (int nj = 0; nj < 4; ++nj) bf[nj] = (sbyte(bw[nj], s) + co) * sb;
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int nj = 0; nj < 4; ++nj)
              cacc[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[mi], bf[nj], cacc[mi][nj], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue.  int32 32x32 C layout: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
  // f64 16x16 layout: col = lane & 15, row = (lane >> 4) + 4 * r.  Each int block goes through a
  // per-wave LDS image so every lane picks up the integer for its f64-layout element.
  __syncthreads();  // staging tiles fully consumed: reuse them as scratch
  int32_t* iscr = reinterpret_cast<int32_t*>(smem) + w * (32 * 33);
  double* tscr = reinterpret_cast<double*>(smem + 4 * 32 * 33 * 4) + w * (16 * 17);
  const bool mirror = tm != tn;
#pragma unroll
  for (int bi = 0; bi < 2; ++bi) {
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
#pragma unroll
      for (int r = 0; r < 16; ++r) iscr[((r & 3) + 8 * (r >> 2) + 4 * h) * 33 + l32] = acc[bi][bj][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int si = 0; si < 2; ++si) {
#pragma unroll
        for (int sj = 0; sj < 2; ++sj) {
          const int mi = 2 * bi + si, nj = 2 * bj + sj;
          const int64_t gj = bn + wc * 64 + nj * 16 + lr;
          const int32_t nbj = gj < n ? Nq[gj] : 0;
          const double cbj = (CORR && gj < n) ? cN[gj] : 0.0;
          double kv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int64_t gi = bm + wr * 64 + mi * 16 + lg + 4 * r;
            const int32_t iv = iscr[(si * 16 + lg + 4 * r) * 33 + sj * 16 + lr];
            const int32_t nai = gi < n ? Nq[gi] : 0;
            const int32_t D = nai + nbj - 2 * iv;  // exact: sum_j (q_aj - q_bj)^2
            double dist = w0 * double(D);
            if (CORR) dist += (gi < n ? cN[gi] : 0.0) + cbj - 2.0 * cacc[mi][nj][r];
            dist = dist > 0.0 ? dist : 0.0;
            kv[r] = exp(neg_gamma * dist);
            if (gi == gj) kv[r] = 1.0;
            if (gi < n && gj < n) K[gi * ldk + gj] = kv[r];
          }
          if (mirror) {
#pragma unroll
            for (int r = 0; r < 4; ++r) tscr[lr * 17 + lg + 4 * r] = kv[r];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int row = lane >> 2, c0 = (lane & 3) * 4;
            const int64_t grow = bn + wc * 64 + nj * 16 + row;
            const int64_t gcol = bm + wr * 64 + mi * 16 + c0;
            if (grow < n) {
              double* dst = K + grow * ldk + gcol;
              const double* sp = tscr + row * 17 + c0;
              if (gcol + 3 < n) {
                *reinterpret_cast<double2*>(dst) = double2{sp[0], sp[1]};
                *reinterpret_cast<double2*>(dst + 2) = double2{sp[2], sp[3]};
              } else {
                for (int q = 0; q < 4; ++q)
                  if (gcol + q < n) dst[q] = sp[q];
              }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

}  // namespace

// Host-side column plan (from the training min/max): which weight is the integer base w0, which
// columns need the FP64 correction, and the permuted column order.
bool plan_quant(const double* mn, const double* mx, int64_t d, QuantPlan* P) {
  P->ok = false;
  if (!mn || !mx || d <= 0) return false;
  std::vector<double> r(static_cast<size_t>(d), 0.0), wgt(static_cast<size_t>(d), 0.0);
  std::map<double, int> freq;
  std::vector<char> live(static_cast<size_t>(d), 0);
  for (int64_t j = 0; j < d; ++j) {
    const double rng = mx[j] - mn[j];
    if (!(rng >= 1e-12)) continue;  // constant column: scaled to 0 everywhere, contributes nothing
    if (rng > 255.0 + 1e-9) return false;
    r[j] = rng;
    wgt[j] = 1.0 / (rng * rng);
    live[j] = 1;
    ++freq[wgt[j]];
  }
  if (freq.empty()) return false;
  double w0 = 0.0;
  int best = -1;
  for (const auto& kv : freq)
    if (kv.second > best) {
      best = kv.second;
      w0 = kv.first;
    }
  std::vector<int32_t> corr, main;
  for (int64_t j = 0; j < d; ++j) {
    if (!live[j]) continue;
    (wgt[j] == w0 ? main : corr).push_back(int32_t(j));
  }
  const int kc = int((corr.size() + 15) / 16 * 16);
  if (kc > kMaxCorr || main.empty()) return false;
  const int kq = int((size_t(kc) + main.size() + QBK - 1) / QBK * QBK);
  P->w0 = w0;
  P->kc = kc;
  P->kq = kq;
  P->perm.assign(size_t(kq), -1);
  P->rmul.assign(size_t(kq), 0.0);
  P->delta.assign(size_t(std::max(kc, 1)), 0.0);
  P->cen.assign(size_t(std::max(kc, 1)), 0.0);
  for (size_t i = 0; i < corr.size(); ++i) {
    P->perm[i] = corr[i];
    P->rmul[i] = r[size_t(corr[i])];
    P->delta[i] = wgt[size_t(corr[i])] - w0;
    P->cen[i] = std::floor(r[size_t(corr[i])] * 0.5);
  }
  for (size_t i = 0; i < main.size(); ++i) {
    P->perm[size_t(kc) + i] = main[i];
    P->rmul[size_t(kc) + i] = r[size_t(main[i])];
  }
  P->n_corr = int(corr.size());
  P->ok = true;
  return true;
}

size_t igram_workspace(int64_t n, const QuantPlan& P) {
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  return al(size_t(n) * size_t(P.kq)) + al(size_t(n) * 4) + al(size_t(n) * 8) + al(size_t(P.kq) * 4) +
         al(size_t(P.kq) * 8) + 2 * al(P.delta.size() * 8) + 256;
}

// Quantise the (scaled) rows and, if every value is an integer multiple of 1/r_j in [0, 255/r_j],
// write the RBF Gram.  Returns SVM_OK with *used = false (nothing written) when the data are not
// integer-valued; ws must hold igram_workspace(n, P) bytes.
int run_igram(hipStream_t s, const double* X, int64_t n, int64_t ld, const QuantPlan& P, double gamma, double* K,
              int64_t ldk, void* ws, bool* used) {
  *used = false;
  if (!P.ok || n <= 0) return SVM_OK;
  if (ldk < n) {
    set_error("igram: ldk < n");
    return SVM_ERR_ARG;
  }
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  char* p = static_cast<char*>(ws);
  int8_t* Q = reinterpret_cast<int8_t*>(p);
  p += al(size_t(n) * size_t(P.kq));
  int32_t* Nq = reinterpret_cast<int32_t*>(p);
  p += al(size_t(n) * 4);
  double* cN = reinterpret_cast<double*>(p);
  p += al(size_t(n) * 8);
  int32_t* perm = reinterpret_cast<int32_t*>(p);
  p += al(size_t(P.kq) * 4);
  double* rmul = reinterpret_cast<double*>(p);
  p += al(size_t(P.kq) * 8);
  double* delta = reinterpret_cast<double*>(p);
  p += al(P.delta.size() * 8);
  double* cen = reinterpret_cast<double*>(p);
  p += al(P.cen.size() * 8);
  unsigned* fail = reinterpret_cast<unsigned*>(p);
  SVMD_CHECK(hipMemcpyAsync(perm, P.perm.data(), P.perm.size() * 4, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(rmul, P.rmul.data(), P.rmul.size() * 8, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(delta, P.delta.data(), P.delta.size() * 8, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(cen, P.cen.data(), P.cen.size() * 8, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemsetAsync(fail, 0, 4, s));
  hipLaunchKernelGGL(quantize_rows_kernel, dim3(unsigned((n + 3) / 4)), dim3(256), 0, s, X, n, ld, perm, rmul,
                     delta, cen, P.kc, P.kq, Q, Nq, cN, fail);
  SVMD_LAUNCH_CHECK();
  unsigned hfail = 1;
  SVMD_CHECK(hipMemcpyAsync(&hfail, fail, 4, hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipStreamSynchronize(s));
  if (hfail) return SVM_OK;  // not integer-valued: caller uses the FP64 path
  const int64_t tiles = (n + QBM - 1) / QBM;
  const int64_t nwg = tiles * (tiles + 1) / 2;
  if (nwg > 0x7FFFFFFF) {
    set_error("igram: problem too large for one launch");
    return SVM_ERR_ARG;
  }
  if (P.kc > 0)
    hipLaunchKernelGGL((igram_tri_kernel<true>), dim3(unsigned(nwg)), dim3(256), 0, s, Q, n, P.kq, P.kc, Nq, cN,
                       delta, cen, P.w0, -gamma, K, ldk, tiles);
  else
    hipLaunchKernelGGL((igram_tri_kernel<false>), dim3(unsigned(nwg)), dim3(256), 0, s, Q, n, P.kq, P.kc, Nq, cN,
                       delta, cen, P.w0, -gamma, K, ldk, tiles);
  SVMD_LAUNCH_CHECK();
  *used = true;
  return SVM_OK;
}

}  // namespace svm355
