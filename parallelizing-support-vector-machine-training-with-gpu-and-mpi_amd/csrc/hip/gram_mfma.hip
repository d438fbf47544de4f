// L2 kernel evaluation on MFMA (gfx950): RBF Gram / cross-kernel blocks in FP64.
//
// Reference: calc_kernel_matrix (gpu_svm_main3.cu:137-147) evaluates ONE kernel row per launch with
// one thread per training point walking a whole 784-double row (uncoalesced, 59 blocks), and the
// SMO loop re-launches it whenever i_high / i_low changes.  Here the full Gram matrix
// (60k^2 FP64 = 28.8 GB, resident in the 288 GB HBM) is produced once by an LDS-tiled
// v_mfma_f64_16x16x4_f64 GEMM X.X^T with the RBF epilogue
//     K_ij = exp(-gamma * max(0, ||x_i||^2 + ||x_j||^2 - 2 x_i.x_j)),   K_ii := 1 (symmetric case)
// so every SMO iteration afterwards only streams two cached rows.
//
// Tiling: 128x128 output tile per 256-thread workgroup, 2x2 waves of 64x64 (4x4 MFMA 16x16
// accumulators per wave, 128 VGPRs of f64 accumulators), BK = 16 doubles per LDS stage with
// register-staged prefetch of the next k-tile while the MFMAs run.  The k index inside a stage is
// permuted (lane group g at sub-step s reads k = 4g + s) so each lane fetches its 4 operands of a
// row with two ds_read_b128; LDS rows are padded to 18 doubles (<= 2-way bank aliasing).
// Workgroup ids are remapped so that consecutive tiles of a GROUP_M x tiles_n band land on one XCD
// (shared L2 for the A row-panel), per the CDNA4 XCD round-robin dispatch.
#include "ctx.h"
#include "tile_map.h"

namespace svm355 {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 16;
constexpr int LS = 18;  // padded LDS row stride (doubles)
constexpr int GROUP_M = 8;

// SYM: force K_ii = 1.  TRI: A == B, compute only tiles tn >= tm and also store each off-diagonal
// tile transposed (staged through LDS so the mirror rows are written as coalesced 32-B runs) —
// half the MFMA work of the full Gram.
template <bool SYM, bool TRI>
__global__ __launch_bounds__(256, 2) void rbf_gram_kernel(
    const double* __restrict__ A, const double* __restrict__ nA, int64_t m, int64_t lda,
    const double* __restrict__ B, const double* __restrict__ nB, int64_t n, int64_t ldb, int64_t kdim,
    double neg_gamma, double* __restrict__ K, int64_t ldk, int64_t tiles_m, int64_t tiles_n,
    const int32_t* __restrict__ gate = nullptr, const int32_t* __restrict__ ncount = nullptr,
    const int32_t* __restrict__ colid = nullptr, int64_t row_off = 0) {
  __shared__ __attribute__((aligned(16))) double As[BM * LS];
  __shared__ __attribute__((aligned(16))) double Bs[BN * LS];
  // Decomposition solver (decomp.hip, FP64 rows): gate = a stopped solve's remaining launches are
  // no-ops; ncount = a device-side bound on the B rows (whole workgroups beyond it exit); colid = B
  // row j is training row colid[j] (A row i is row_off + i): that pair's value is the diagonal, 1.
  if (gate && *gate != 0) return;
  if (ncount) n = std::min<int64_t>(n, int64_t(*ncount));

  int64_t tm, tn;
  if (TRI) {
    const int64_t nwg = tiles_m * (tiles_m + 1) / 2;
    tri_tile(xcd_remap(blockIdx.x, nwg), tiles_m, tm, tn);
  } else {
    const int64_t nwg = tiles_m * tiles_n;
    const int64_t wg = xcd_remap(blockIdx.x, nwg);
    const int64_t band = GROUP_M * tiles_n;
    const int64_t first_m = (wg / band) * GROUP_M;
    const int64_t gsz = std::min<int64_t>(tiles_m - first_m, GROUP_M);
    tm = first_m + (wg % band) % gsz;
    tn = (wg % band) / gsz;
  }
  const int64_t bm = tm * BM, bn = tn * BN;
  if (ncount && bn >= n) return;

  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int lr = lane & 15, lg = lane >> 4;

  // Staging: thread t copies 8 consecutive doubles (4 x 16 B) of tile row t>>1.
  const int srow = t >> 1, scol = (t & 1) * 8;
  const bool aok = bm + srow < m, bok = bn + srow < n;
  const double* ap = A + (aok ? (bm + srow) * lda : 0) + scol;
  const double* bp = B + (bok ? (bn + srow) * ldb : 0) + scol;
  double2 ra[4], rb[4];
  const double2 z2 = {0.0, 0.0};
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = aok ? *reinterpret_cast<const double2*>(ap + k0 + 2 * i) : z2;
      rb[i] = bok ? *reinterpret_cast<const double2*>(bp + k0 + 2 * i) : z2;
    }
  };
  gload(0);

  f64x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f64x4{0.0, 0.0, 0.0, 0.0};

  for (int64_t k0 = 0; k0 < kdim; k0 += BK) {
    __syncthreads();  // previous stage fully consumed
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<double2*>(&As[srow * LS + scol + 2 * i]) = ra[i];
      *reinterpret_cast<double2*>(&Bs[srow * LS + scol + 2 * i]) = rb[i];
    }
    __syncthreads();
    if (k0 + BK < kdim) gload(k0 + BK);  // overlaps the MFMAs below

    double a[4][4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const double* p = &As[(wr * 64 + mi * 16 + lr) * LS + 4 * lg];
      const double2 x0 = *reinterpret_cast<const double2*>(p);
      const double2 x1 = *reinterpret_cast<const double2*>(p + 2);
      a[mi][0] = x0.x;
      a[mi][1] = x0.y;
      a[mi][2] = x1.x;
      a[mi][3] = x1.y;
    }
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
      const double* p = &Bs[(wc * 64 + nj * 16 + lr) * LS + 4 * lg];
      const double2 y0 = *reinterpret_cast<const double2*>(p);
      const double2 y1 = *reinterpret_cast<const double2*>(p + 2);
      const double b[4] = {y0.x, y0.y, y1.x, y1.y};
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          acc[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi][s], b[s], acc[mi][nj], 0, 0, 0);
    }
  }

  // Epilogue: f64 16x16x4 C/D layout is col = lane & 15, row = (lane >> 4) + 4 * reg.
  double nb[4], na[4][4];
#pragma unroll
  for (int nj = 0; nj < 4; ++nj) {
    const int64_t gj = bn + wc * 64 + nj * 16 + lr;
    nb[nj] = gj < n ? nB[gj] : 0.0;
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t gi = bm + wr * 64 + mi * 16 + lg + 4 * r;
      na[mi][r] = gi < m ? nA[gi] : 0.0;
    }
  const bool mirror = TRI && tm != tn;
  double* scr = As + w * (16 * 17);  // per-wave 16x16 transpose buffer (+1 pad)
  if (mirror) __syncthreads();       // every wave is done reading the k-loop's LDS tiles
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
      const int64_t gj = bn + wc * 64 + nj * 16 + lr;
      double kv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gi = bm + wr * 64 + mi * 16 + lg + 4 * r;
        double dist = na[mi][r] + nb[nj] - 2.0 * acc[mi][nj][r];
        dist = dist > 0.0 ? dist : 0.0;
        kv[r] = exp(neg_gamma * dist);
        if (SYM && gi == gj) kv[r] = 1.0;
        if (!SYM && colid && gj < n && gi + row_off == int64_t(colid[gj])) kv[r] = 1.0;
        if (gi < m && gj < n) K[gi * ldk + gj] = kv[r];
      }
      if (mirror) {
        // Transpose the 16x16 sub-tile through LDS: scr[c][r] = tile[r][c].
#pragma unroll
        for (int r = 0; r < 4; ++r) scr[lr * 17 + lg + 4 * r] = kv[r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int row = lane >> 2, c0 = (lane & 3) * 4;
        const int64_t grow = bn + wc * 64 + nj * 16 + row;      // mirrored row  (an original column)
        const int64_t gcol = bm + wr * 64 + mi * 16 + c0;       // mirrored cols (original rows)
        if (grow < n) {
          double* dst = K + grow * ldk + gcol;
          const double* s = scr + row * 17 + c0;
          if (gcol + 3 < m) {
            *reinterpret_cast<double2*>(dst) = double2{s[0], s[1]};
            *reinterpret_cast<double2*>(dst + 2) = double2{s[2], s[3]};
          } else {
            for (int q = 0; q < 4; ++q)
              if (gcol + q < m) dst[q] = s[q];
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  }
}

// out[i] = sum_k coef[k] * K[i][k] - b; one wave per row, fixed butterfly order (deterministic).
__global__ __launch_bounds__(256) void gemv_rows_kernel(const double* __restrict__ K, int64_t ldk,
                                                        int64_t m, int64_t n,
                                                        const double* __restrict__ coef, double b,
                                                        double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= m) return;
  const double* kr = K + row * ldk;
  double acc = 0.0;
  for (int64_t k = lane; k < n; k += 64) acc += coef[k] * kr[k];
  acc = wave_sum(acc);
  if (lane == 0) out[row] = acc - b;
}

// Accuracy epilogue of prediction (the reference's predict flag + reduce_sum, gpu_svm_main3.cu:277-315,
// which sums 0/1 doubles in a multi-pass tree): count rows whose sign matches the label, integer
// wave sums and one atomic per wave.  zero_positive: s >= 0 -> +1 (cascade rule, M3 :800), else s > 0.
__global__ __launch_bounds__(256) void count_correct_kernel(const double* __restrict__ dec,
                                                            const int32_t* __restrict__ y, int64_t m,
                                                            int zero_positive,
                                                            unsigned long long* __restrict__ count) {
  unsigned c = 0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    const double s = dec[i];
    const int pred = (zero_positive ? s >= 0.0 : s > 0.0) ? 1 : -1;
    c += pred == y[i] ? 1u : 0u;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, (unsigned long long)c);
}

}  // namespace

int count_correct(DeviceCtx* ctx, const double* dec, const int32_t* y, int64_t m, bool zero_positive,
                  int64_t* out) {
  *out = 0;
  if (m <= 0) return SVM_OK;
  hipStream_t s = ctx->stream;
  if (!ctx->count_d) SVMD_CHECK(hipMalloc(&ctx->count_d, 1024 * 8));
  int rc = ctx->ensure_pinned(8);
  if (rc) return rc;
  SVMD_CHECK(hipMemsetAsync(ctx->count_d, 0, 8, s));
  const unsigned bx = unsigned(std::min<int64_t>((m + 255) / 256, 1024));
  hipLaunchKernelGGL(count_correct_kernel, dim3(bx), dim3(256), 0, s, dec, y, m, zero_positive ? 1 : 0,
                     static_cast<unsigned long long*>(ctx->count_d));
  SVMD_LAUNCH_CHECK();
  auto* h = static_cast<unsigned long long*>(ctx->pinned);
  SVMD_CHECK(hipMemcpyAsync(h, ctx->count_d, 8, hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipStreamSynchronize(s));
  *out = int64_t(h[0]);
  return SVM_OK;
}

int launch_rbf_gram(hipStream_t s, const double* A, const double* nA, int64_t m, int64_t lda,
                    const double* B, const double* nB, int64_t n, int64_t ldb, int64_t kdim,
                    double gamma, double* K, int64_t ldk, bool sym_diag) {
  if (m <= 0 || n <= 0) return SVM_OK;
  if (kdim % BK || lda < kdim || ldb < kdim || ldk < n || (lda % 2) || (ldb % 2) ||
      (reinterpret_cast<uintptr_t>(A) & 15) || (reinterpret_cast<uintptr_t>(B) & 15)) {
    set_error("rbf_gram: kdim must be a multiple of %d, lda/ldb even and >= kdim, ldk >= n, "
              "A/B 16-byte aligned (kdim=%lld lda=%lld ldb=%lld ldk=%lld n=%lld)",
              BK, (long long)kdim, (long long)lda, (long long)ldb, (long long)ldk, (long long)n);
    return SVM_ERR_ARG;
  }
  const int64_t tiles_m = (m + BM - 1) / BM, tiles_n = (n + BN - 1) / BN;
  const int64_t nwg = tiles_m * tiles_n;
  if (nwg > 0x7FFFFFFF) {
    set_error("rbf_gram: problem too large for one launch");
    return SVM_ERR_ARG;
  }
  const char* tv = getenv("SVM355_GRAM_TRI");
  const bool tri = sym_diag && A == B && nA == nB && m == n && lda == ldb && !(tv && tv[0] == '0');
  if (tri)
    hipLaunchKernelGGL((rbf_gram_kernel<true, true>), dim3(unsigned(tiles_m * (tiles_m + 1) / 2)), dim3(256), 0, s,
                       A, nA, m, lda, B, nB, n, ldb, kdim, -gamma, K, ldk, tiles_m, tiles_n);
  else if (sym_diag)
    hipLaunchKernelGGL((rbf_gram_kernel<true, false>), dim3(unsigned(nwg)), dim3(256), 0, s, A, nA, m, lda, B, nB,
                       n, ldb, kdim, -gamma, K, ldk, tiles_m, tiles_n);
  else
    hipLaunchKernelGGL((rbf_gram_kernel<false, false>), dim3(unsigned(nwg)), dim3(256), 0, s, A, nA, m, lda, B, nB,
                       n, ldb, kdim, -gamma, K, ldk, tiles_m, tiles_n);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

int launch_rbf_block_dev(hipStream_t s, const double* A, const double* nA, int64_t m, int64_t lda, const double* B,
                         const double* nB, int64_t ncap, int64_t ldb, int64_t kdim, double gamma, double* K, int64_t ldk,
                         bool sym_diag, const int32_t* gate, const int32_t* ncount, const int32_t* colid,
                         int64_t row_off) {
  if (m <= 0 || ncap <= 0) return SVM_OK;
  if (kdim % BK || lda < kdim || ldb < kdim || ldk < ncap || (lda % 2) || (ldb % 2) ||
      (reinterpret_cast<uintptr_t>(A) & 15) || (reinterpret_cast<uintptr_t>(B) & 15)) {
    set_error("rbf block: kdim must be a multiple of %d, lda/ldb even and >= kdim, ldk >= ncap, A/B 16-byte aligned",
              BK);
    return SVM_ERR_ARG;
  }
  const int64_t tiles_m = (m + BM - 1) / BM, tiles_n = (ncap + BN - 1) / BN;
  const int64_t nwg = tiles_m * tiles_n;
  if (nwg > 0x7FFFFFFF) {
    set_error("rbf block: problem too large for one launch");
    return SVM_ERR_ARG;
  }
  if (sym_diag)
    hipLaunchKernelGGL((rbf_gram_kernel<true, false>), dim3(unsigned(nwg)), dim3(256), 0, s, A, nA, m, lda, B, nB,
                       ncap, ldb, kdim, -gamma, K, ldk, tiles_m, tiles_n, gate, ncount, colid, row_off);
  else
    hipLaunchKernelGGL((rbf_gram_kernel<false, false>), dim3(unsigned(nwg)), dim3(256), 0, s, A, nA, m, lda, B, nB,
                       ncap, ldb, kdim, -gamma, K, ldk, tiles_m, tiles_n, gate, ncount, colid, row_off);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

int launch_gemv_rows(hipStream_t s, const double* K, int64_t ldk, int64_t m, int64_t n,
                     const double* coef, double b, double* out) {
  if (m <= 0) return SVM_OK;
  hipLaunchKernelGGL(gemv_rows_kernel, dim3(unsigned((m + 3) / 4)), dim3(256), 0, s, K, ldk, m, n, coef,
                     b, out);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

}  // namespace svm355

SVMD_TU_WARM(gram_mfma)
