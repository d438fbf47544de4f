// L2 kernel evaluation, exact-integer path: RBF Gram of integer-valued features on int8 MFMA.
//
// MNIST-shaped inputs are integer pixel intensities, and after the reference's min-max scaling
// (main3.cpp:74-89) feature j of every row is x_j = q_j / r_j with q_j = p_j - min_j an integer in
// [0, r_j] and r_j = max_j - min_j <= 255.  Grouping the columns by range (weight w_g = 1 / r_g^2):
//
//     ||x_a - x_b||^2 = sum_g w_g sum_{j in g} (q_aj - q_bj)^2
//
// Every column is stored as ONE signed byte, centred on ceil(r_j / 2) (differences are invariant
// to the shift), and every group's cross term I_g = sum_{j in g} q'_aj q'_bj is an exact int32
// v_mfma_i32_32x32x32_i8 accumulation:
//   * the MAIN group (the most common range: r = 255 on MNIST) is accumulated last and kept as an
//     integer: D0 = N0_a + N0_b - 2 I0 is the EXACT integer sum of squared differences;
//   * every other group ("extra" columns, each group padded to a 32-column k-step) is flushed at
//     its last k-step into an FP64 accumulator X += w_g * I_g that lives in the same 32x32
//     accumulator layout (no lane shuffles), with per-row weighted norms WN = sum w_g N_g.
// dist = w0 * D0 + (WN_a + WN_b - 2 X): the dominant part is exact, the extra part is small
// (centred operands), so every kernel value is FP64-accurate (tests/test_gpu_kernels.py checks
// |K - K_exact| <= 2e-15) and the Gram is exactly symmetric.  No FP64 MFMA work remains.
//
// Reference: calc_kernel_matrix (gpu_svm_main3.cu:137-147) evaluates one FP64 row per launch with
// a d-long scalar loop per thread.  Here the whole upper-triangular Gram is produced in one launch
// (128x128 tiles split into two 128x64 workgroups of 4 waves x 32x64 = 2 MFMA 32x32 tiles per
// wave, XCD-aware tile order) and the mirror half is written through a per-wave LDS transpose.
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
typedef double f64x2 __attribute__((ext_vector_type(2)));

constexpr int QBM = 128;        // tile rows
constexpr int QBN = 64;         // columns per workgroup (half of a 128x128 tile)
constexpr int kMaxSteps = 128;  // 32-column k-steps (kq <= 4096)
constexpr int kColAlign = 128;  // kq is a multiple of this (host plan): 128-column LDS stages
// LDS: per-tile tables (step weights, row/col norms) first, then a union of the int8 staging tiles
// (k-loop) and the per-wave 32x33 f64 transpose images (epilogue).
constexpr int kTableBytes = kMaxSteps * 8 + (QBM + QBN) * 12;
constexpr int kImgBytes = 4 * 32 * 33 * 8;
template <int BK>
struct IgramCfg {
  static constexpr int LS = BK + 16;  // row stride in bytes: conflict-free ds_read_b128 for BK = 64 / 128
  static constexpr int kStage = (QBM + QBN) * LS;
  static constexpr int kUnion = kStage > kImgBytes ? kStage : kImgBytes;
  static constexpr int kSmem = kTableBytes + kUnion;
};

// ---- quantisation: one wave per row.  Writes the permuted centred int8 row q'_k = q_k - off_k,
// N0 = sum_{main} q'^2 (exact int) and WN = sum_{extra} w_k q'^2; flags any value that is not an
// integer in [0, 255] (the caller then uses the FP64 Gram).
__global__ __launch_bounds__(256) void quantize_rows_kernel(
    const double* __restrict__ X, int64_t n, int64_t ld, const int32_t* __restrict__ perm,
    const double* __restrict__ rmul, const double* __restrict__ off, const double* __restrict__ wx, int main0,
    int kq, int8_t* __restrict__ Q, int32_t* __restrict__ N0, double* __restrict__ WN, unsigned* __restrict__ fail) {
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const double* xr = X + row * ld;
  int32_t* qr = reinterpret_cast<int32_t*>(Q + row * int64_t(kq));
  int32_t nacc = 0;
  double wacc = 0.0;
  bool bad = false;
  for (int w = lane; w < kq / 4; w += 64) {
    uint32_t word = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int k = 4 * w + b;
      const int j = perm[k];
      int qq = 0;
      if (j >= 0) {
        // x = q / r rounded once, so x * r recovers the integer q to within 2 ulp(q) <= 6e-14;
        // anything farther off is not an integer pixel (e.g. 3.0000004) and takes the FP64 Gram.
        const double v = xr[j] * rmul[k];
        const double q = rint(v);
        bad |= !(fabs(v - q) <= 64.0 * __DBL_EPSILON__ * fmax(1.0, rmul[k])) || q < 0.0 || q > 255.0;
        qq = int(q - off[k]);
        if (k >= main0)
          nacc += qq * qq;
        else
          wacc += wx[k] * double(qq * qq);
      }
      word |= uint32_t(uint8_t(int8_t(qq))) << (8 * b);
    }
    qr[w] = int32_t(word);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nacc += __shfl_xor(nacc, o, kWave);
  wacc = wave_sum(wacc);
  if (lane == 0) {
    N0[row] = nacc;
    WN[row] = wacc;
  }
  if (__any(bad) && lane == 0) atomicOr(fail, 1u);
}

// Same quantisation with the column tables staged once per workgroup in LDS (perm; range and offset
// as one packed int32 -- both are small integers, exact as doubles; the extra-group weights) and the
// workgroup walking many rows: the per-element table loads of quantize_rows_kernel become LDS reads.
// Every lane handles the same k in the same order with the same arithmetic, so N0 / WN / Q are
// bit-identical.  kq <= kQuantLdsMaxKq.
constexpr int kQuantLdsMaxKq = 32 * kMaxSteps;  // tables <= 64 KB of LDS
__global__ __launch_bounds__(256) void quantize_rows_lds_kernel(
    const double* __restrict__ X, int64_t n, int64_t ld, const int32_t* __restrict__ perm,
    const double* __restrict__ rmul, const double* __restrict__ off, const double* __restrict__ wx, int main0,
    int kq, int8_t* __restrict__ Q, int32_t* __restrict__ N0, double* __restrict__ WN, unsigned* __restrict__ fail) {
  extern __shared__ __attribute__((aligned(16))) char qsm[];
  int32_t* sp = reinterpret_cast<int32_t*>(qsm);
  int32_t* sro = sp + kq;
  double* swx = reinterpret_cast<double*>(sro + kq);
  for (int k = threadIdx.x; k < kq; k += 256) {
    sp[k] = perm[k];
    sro[k] = int32_t(rmul[k]) | (int32_t(off[k]) << 16);
    if (k < main0) swx[k] = wx[k];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  bool bad = false;
  for (int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); row < n; row += int64_t(gridDim.x) * 4) {
    const double* xr = X + row * ld;
    int32_t* qr = reinterpret_cast<int32_t*>(Q + row * int64_t(kq));
    int32_t nacc = 0;
    double wacc = 0.0;
    for (int w = lane; w < kq / 4; w += 64) {
      uint32_t word = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int k = 4 * w + b;
        const int j = sp[k];
        int qq = 0;
        if (j >= 0) {
          const int32_t ro = sro[k];
          const double rk = double(ro & 0xFFFF), ok = double(ro >> 16);
          const double v = xr[j] * rk;
          const double q = rint(v);
          bad |= !(fabs(v - q) <= 64.0 * __DBL_EPSILON__ * fmax(1.0, rk)) || q < 0.0 || q > 255.0;
          qq = int(q - ok);
          if (k >= main0)
            nacc += qq * qq;
          else
            wacc += swx[k] * double(qq * qq);
        }
        word |= uint32_t(uint8_t(int8_t(qq))) << (8 * b);
      }
      qr[w] = int32_t(word);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nacc += __shfl_xor(nacc, o, kWave);
    wacc = wave_sum(wacc);
    if (lane == 0) {
      N0[row] = nacc;
      WN[row] = wacc;
    }
  }
  if (__any(bad) && lane == 0) atomicOr(fail, 1u);
}

// Quantisation straight from the uint8 pixel rows (n x d, contiguous) -- no FP64 rows at all.  For a
// column j of range r_j in a group of range R (r_j divides R), the FP64 path rounds
// ((p - mn_j) / r_j) * R to the integer (p - mn_j) * (R / r_j); this kernel forms that integer
// directly, so Q, N0 and WN are bit-identical (same k per lane, same accumulation order).  Tables:
// perm, one packed int32 per k (mn_j | R / r_j << 8 | offset << 16), the extra-group weights.
__global__ __launch_bounds__(256) void quantize_u8_lds_kernel(
    const uint8_t* __restrict__ Xu, int64_t n, int64_t d, const int32_t* __restrict__ perm,
    const int32_t* __restrict__ pack, const double* __restrict__ wx, int main0, int kq, int8_t* __restrict__ Q,
    int32_t* __restrict__ N0, double* __restrict__ WN, unsigned* __restrict__ fail) {
  extern __shared__ __attribute__((aligned(16))) char qsm[];
  int32_t* sp = reinterpret_cast<int32_t*>(qsm);
  int32_t* spk = sp + kq;
  double* swx = reinterpret_cast<double*>(spk + kq);
  for (int k = threadIdx.x; k < kq; k += 256) {
    sp[k] = perm[k];
    spk[k] = pack[k];
    if (k < main0) swx[k] = wx[k];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  bool bad = false;
  for (int64_t row = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); row < n; row += int64_t(gridDim.x) * 4) {
    const uint8_t* xr = Xu + row * d;
    int32_t* qr = reinterpret_cast<int32_t*>(Q + row * int64_t(kq));
    int32_t nacc = 0;
    double wacc = 0.0;
    for (int w = lane; w < kq / 4; w += 64) {
      uint32_t word = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int k = 4 * w + b;
        const int j = sp[k];
        int qq = 0;
        if (j >= 0) {
          const int32_t pk = spk[k];
          const int q = (int(xr[j]) - (pk & 0xFF)) * ((pk >> 8) & 0xFF);
          bad |= q < 0 || q > 255;
          qq = q - (pk >> 16);
          if (k >= main0)
            nacc += qq * qq;
          else
            wacc += swx[k] * double(qq * qq);
        }
        word |= uint32_t(uint8_t(int8_t(qq))) << (8 * b);
      }
      qr[w] = int32_t(word);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nacc += __shfl_xor(nacc, o, kWave);
    wacc = wave_sum(wacc);
    if (lane == 0) {
      N0[row] = nacc;
      WN[row] = wacc;
    }
  }
  if (__any(bad) && lane == 0) atomicOr(fail, 1u);
}

// ---- exp over a batch of lanes' values, bit-identical to the device libm exp (same operation
// sequence: x*log2e, round-to-even, two-part ln2 reduction, degree-11 polynomial in 12 FMAs,
// ldexp, overflow/underflow clamps).  Evaluating B values per coefficient lets one VGPR copy of
// each 64-bit coefficient serve all B FMAs; a scalar libm call reloads all twelve per value
// (two v_mov each), which made v_mov the most frequent instruction of the Gram kernel.
__device__ __forceinline__ constexpr double hexd(uint64_t u) { return __builtin_bit_cast(double, u); }
// d = a * b + c with the wave-uniform c read from an SGPR pair (VOP3 src2): the compiler would
// otherwise copy the constant into the tied destination of v_fmac_f64 before every use.
__device__ __forceinline__ double fma_s(double a, double b, double c) {
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
  return d;
}
template <int B>
__device__ __forceinline__ void exp_batch(double (&x)[B]) {
  constexpr double kC[10] = {hexd(0x3ec71dee623fde64ull), hexd(0x3efa01997c89e6b0ull), hexd(0x3f2a01a014761f6eull),
                             hexd(0x3f56c16c1852b7b0ull), hexd(0x3f81111111122322ull), hexd(0x3fa55555555502a1ull),
                             hexd(0x3fc5555555555511ull), hexd(0x3fe000000000000bull), 1.0, 1.0};
  double n[B], r[B], p[B];
#pragma unroll
  for (int i = 0; i < B; ++i) n[i] = __builtin_rint(x[i] * hexd(0x3ff71547652b82feull));
#pragma unroll
  for (int i = 0; i < B; ++i) r[i] = __builtin_fma(hexd(0xbfe62e42fefa39efull), n[i], x[i]);
#pragma unroll
  for (int i = 0; i < B; ++i) r[i] = __builtin_fma(hexd(0xbc7abc9e3b39803full), n[i], r[i]);
#pragma unroll
  for (int i = 0; i < B; ++i) p[i] = fma_s(hexd(0x3e5ade156a5dcb37ull), r[i], hexd(0x3e928af3fca7ab0cull));
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int i = 0; i < B; ++i) p[i] = fma_s(r[i], p[i], kC[c]);
#pragma unroll
  for (int c = 8; c < 10; ++c)  // + 1.0 twice: an inline constant
#pragma unroll
    for (int i = 0; i < B; ++i) p[i] = __builtin_fma(r[i], p[i], kC[c]);
#pragma unroll
  for (int i = 0; i < B; ++i) {
    double e = __builtin_ldexp(p[i], int(n[i]));
    e = x[i] > 1024.0 ? __builtin_inf() : e;
    x[i] = x[i] < -1075.0 ? 0.0 : e;
  }
}

// Self-test hook: out_lib[i] = exp(x[i]) (device libm), out_batch[i] = exp_batch (8 per lane).
__global__ __launch_bounds__(256) void exp_check_kernel(const double* __restrict__ x, int64_t n,
                                                        double* __restrict__ out_lib,
                                                        double* __restrict__ out_batch) {
  const int64_t base = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) * 8;
  double v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = base + i < n ? x[base + i] : 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (base + i < n) out_lib[base + i] = exp(v[i]);
  exp_batch<8>(v);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (base + i < n) out_batch[base + i] = v[i];
}

// Upper-triangular 128x128 tiles of K = exp(-gamma * dist), each split into two 128x64 halves
// (one workgroup each: 4 waves x 32 rows x 64 columns, 2 MFMA 32x32 tiles per wave), each
// off-diagonal tile also stored transposed.  kq = int8 columns (multiple of BK); columns
// [0, main0) are the extra groups (main0 a multiple of 32), step_w[s] = weight of k-step s's group
// if s is the LAST k-step of its group (flush), else 0.  BK = int8 columns per LDS stage.
// RECT: the block K(rows [0, n), rows [col0, col0 + ncols)) of the same quantised set instead of the
// symmetric Gram (every 128 x 128 tile of the tiles x ctiles grid, no mirror; column j of the block
// at K[i * ldk + j]), e.g. the kernel values of a training set against its leading support vectors
// (the cascade's warm-start check) or a distributed-SMO team's slab K(:, own) (dsmo.hip).
//
// GEMV (RECT only, decomposition solver, decomp.hip): block column j is row colid[j] of the same
// quantised set, for j < *ncount (a device-side count: workgroups whose 64 columns all lie beyond it
// exit at once), and instead of storing K the epilogue writes, per row, the sum over this
// workgroup's 64 columns of coef[j] * K(row, colid[j]) to K[row * ldk + (column-half index)] (a
// fixed-order butterfly: the caller adds the halves in index order, so the f update is
// deterministic).
// CST (with GEMV, decomposition column cache): the same columns and kernel values, stored instead of
// reduced: K(row, colid[j]) to K[slot[j] * ldk + row] (column j's cache slot, rows contiguous).
// diag (GEMV / CST, optional): the row operand is a packed subset of the rows (a shrunk solve's active
// rows, decomp.hip) and column j's point is row diag[j] of it (-1: none) -- the unit diagonal is then
// local row == diag[j] (row_off 0) instead of row_off + row == colid[j].
template <bool EXTRA, int BK, bool RECT = false, bool GEMV = false, bool CST = false>
__global__ __launch_bounds__(256, 2) void igram_tri_kernel(
    const int8_t* __restrict__ Q, int64_t n, int kq, int main0, const int32_t* __restrict__ N0,
    const double* __restrict__ WN, const double* __restrict__ step_w, double w0, double neg_gamma,
    double* __restrict__ K, int64_t ldk, int64_t tiles, int64_t ncols, int64_t col0 = 0,
    const int32_t* __restrict__ colid = nullptr, const double* __restrict__ coef = nullptr,
    const int32_t* __restrict__ ncount = nullptr, const int8_t* __restrict__ Qc = nullptr,
    const int32_t* __restrict__ N0c = nullptr, const double* __restrict__ WNc = nullptr, int64_t row_off = 0,
    const int32_t* __restrict__ gate = nullptr, int64_t cstride = 0, const int32_t* __restrict__ slot = nullptr,
    const int32_t* __restrict__ diag = nullptr) {
  static_assert(!GEMV || RECT, "the GEMV epilogue is a rectangular block's");
  static_assert(!CST || GEMV, "the column store is the GEMV's operands with a store epilogue");
  if (gate && *gate != 0) return;  // a stopped decomposition solve's remaining batch (decomp.hip)
  using Cfg = IgramCfg<BK>;
  constexpr int QLS = Cfg::LS;
  constexpr int CPR = BK / 16;            // 16-byte chunks per staged row
  constexpr int RPP = 256 / CPR;          // rows per staging pass
  constexpr int APASS = QBM / RPP, BPASS = QBN / RPP;
  __shared__ __attribute__((aligned(16))) char smem[Cfg::kSmem];
  double* sw = reinterpret_cast<double*>(smem);
  double* wn_r = sw + kMaxSteps;                     // WN of the tile's 128 rows / 64 cols
  double* wn_c = wn_r + QBM;
  int32_t* n0_r = reinterpret_cast<int32_t*>(wn_c + QBN);
  int32_t* n0_c = n0_r + QBM;
  char* As = smem + kTableBytes;                     // 128 rows x QLS
  char* Bs = As + QBM * QLS;                         // 64 rows x QLS
  double* img = reinterpret_cast<double*>(smem + kTableBytes);  // epilogue: per-wave 32x33 images

  const int64_t ctiles = RECT ? (ncols + QBM - 1) / QBM : tiles;
  const int64_t c0 = RECT ? col0 : 0;      // global row index of block column 0
  // column operand: the same rows, or for GEMV the full set the ids colid index (the row operand may
  // be a slice of it starting at global row row_off)
  const int8_t* __restrict__ Qb = GEMV ? Qc : Q;
  const int32_t* __restrict__ N0b = GEMV ? N0c : N0;
  const double* __restrict__ WNb = GEMV ? WNc : WN;
  const int64_t ntile = RECT ? tiles * ctiles : tiles * (tiles + 1) / 2;
  // GEMV with cstride == QBN: one workgroup per row tile walks every column half
  const bool walk_all = GEMV && cstride == QBN;
  const int64_t wg = xcd_remap(blockIdx.x, walk_all ? tiles : 2 * ntile);
  int64_t tm, tn;
  if (walk_all) {
    tm = wg;
    tn = 0;
  } else if (RECT) {
    tm = (wg >> 1) / ctiles;
    tn = (wg >> 1) - tm * ctiles;
  } else {
    tri_tile(wg >> 1, tiles, tm, tn);
  }
  const int64_t bm_ = tm * QBM;
  int64_t bn = tn * QBM + (walk_all ? 0 : (wg & 1) * QBN);
  // column bound (block-local); GEMV: the device-side count, whole workgroups beyond it exit
  const int64_t ncol = GEMV ? int64_t(*ncount) : RECT ? ncols : n;
  // global row of block column j: c0 + j, or colid[j] (GEMV)
  auto crow = [&](int64_t j) -> int64_t { return GEMV ? int64_t(colid[j]) : c0 + j; };
  // GEMV with cstride > 0: the grid covers ncols columns per row tile and each workgroup walks its
  // half, then the halves cstride columns further on, up to *ncount (few workgroups exit unused)
  for (;;) {
  if (GEMV && bn >= ncol) return;
  // opaque per pass: nothing derived from the row tile is hoisted out of the GEMV loop (that held
  // its addresses live across the whole k-loop and spilled)
  int64_t bm = bm_;
  if constexpr (GEMV) asm volatile("" : "+s"(bm));
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int main_step0 = main0 / 32;
  if (EXTRA)
    for (int k = t; k < main_step0; k += 256) sw[k] = step_w[k];
  if (t < QBM) {
    const int64_t gi = bm + t;
    n0_r[t] = gi < n ? N0[gi] : 0;
    if (EXTRA) wn_r[t] = gi < n ? WN[gi] : 0.0;
  } else if (t < QBM + QBN) {
    const int64_t gj = bn + (t - QBM);
    n0_c[t - QBM] = gj < ncol ? N0b[crow(gj)] : 0;
    if (EXTRA) wn_c[t - QBM] = gj < ncol ? WNb[crow(gj)] : 0.0;
  }

  // Staging per BK-column stage: thread t copies 16-byte chunk t % CPR of rows t / CPR + RPP * p.
  const int srow = t / CPR, scol = (t % CPR) * 16;
  const i32x4 zero4 = {0, 0, 0, 0};
  i32x4 ga[APASS], gb[BPASS];
  int64_t brow[BPASS];  // global rows of this thread's staged B rows (-1: beyond the block)
#pragma unroll
  for (int p = 0; p < BPASS; ++p) {
    const int64_t r = bn + srow + RPP * p;
    brow[p] = r < (RECT ? ncol : n) ? crow(r) : -1;
  }
  auto gload = [&](int k0) {
#pragma unroll
    for (int p = 0; p < APASS; ++p) {
      const int64_t r = bm + srow + RPP * p;
      ga[p] = r < n ? *reinterpret_cast<const i32x4*>(Q + r * kq + k0 + scol) : zero4;
    }
#pragma unroll
    for (int p = 0; p < BPASS; ++p)
      gb[p] = brow[p] >= 0 ? *reinterpret_cast<const i32x4*>(Qb + brow[p] * kq + k0 + scol) : zero4;
  };
  gload(0);

  i32x16 acc[2];
  double xacc[2][16];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc[j][r] = 0;
      if (EXTRA) xacc[j][r] = 0.0;
    }

  // After an extra group's flush the next k-step starts its accumulators from the inline constant 0
  // (an MFMA operand) instead of zeroing 32 registers per lane with v_mov.
  bool fresh = false;
  const i32x16 zero16 = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int k0 = 0; k0 < kq; k0 += BK) {
    __syncthreads();
#pragma unroll
    for (int p = 0; p < APASS; ++p) *reinterpret_cast<i32x4*>(As + (srow + RPP * p) * QLS + scol) = ga[p];
#pragma unroll
    for (int p = 0; p < BPASS; ++p) *reinterpret_cast<i32x4*>(Bs + (srow + RPP * p) * QLS + scol) = gb[p];
    __syncthreads();
    if (k0 + BK < kq) gload(k0 + BK);

    // A and B fragments use the same (lane, byte) -> k map, so the product is independent of the
    // hardware's k order inside a step.
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const i32x4 a = *reinterpret_cast<const i32x4*>(As + (w * 32 + l32) * QLS + ks * 32 + 16 * h);
      i32x4 b[2];
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
        b[nj] = *reinterpret_cast<const i32x4*>(Bs + (nj * 32 + l32) * QLS + ks * 32 + 16 * h);
      if (EXTRA && fresh) {
#pragma unroll
        for (int nj = 0; nj < 2; ++nj) acc[nj] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b[nj], zero16, 0, 0, 0);
        fresh = false;
      } else {
#pragma unroll
        for (int nj = 0; nj < 2; ++nj) acc[nj] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b[nj], acc[nj], 0, 0, 0);
      }
      if (EXTRA) {
        const int step = k0 / 32 + ks;
        if (step < main_step0) {
          const double wgt = sw[step];
          if (wgt != 0.0) {  // last k-step of an extra group: flush its exact cross term
#pragma unroll
            for (int nj = 0; nj < 2; ++nj)
#pragma unroll
              for (int r = 0; r < 16; ++r) xacc[nj][r] = __builtin_fma(wgt, double(acc[nj][r]), xacc[nj][r]);
            fresh = true;
          }
        }
      }
    }
  }

  __syncthreads();  // staging tiles fully consumed: the union becomes the transpose images
  if constexpr (CST) {
    // ---- column-store epilogue: the GEMV's kernel values (the same arithmetic, bit for bit) to the
    // columns' cache slots; a lane's four consecutive rows are 32 contiguous bytes of one slot
    const int64_t row0 = bm + w * 32 + 4 * h;
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
      const int cl = bj * 32 + l32;
      const int64_t gj = bn + cl;
      const bool colok = gj < ncol;
      const int64_t gid = colok ? int64_t(diag ? diag[gj] : colid[gj]) : -1;
      double* dst = K + (colok ? int64_t(slot[gj]) * ldk : 0);
      const int32_t nbj = n0_c[cl];
      const double wbj = EXTRA ? wn_c[cl] : 0.0;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        double ex[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int r = 8 * half + q;
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
          const int32_t D0 = n0_r[w * 32 + rl] + nbj - 2 * acc[bj][r];
          double dist = w0 * double(D0);
          if (EXTRA) dist += (wn_r[w * 32 + rl] + wbj) - 2.0 * xacc[bj][r];
          dist = dist > 0.0 ? dist : 0.0;
          ex[q] = neg_gamma * dist;
        }
        exp_batch<8>(ex);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int r = 8 * half + q;
          const int64_t gi = row0 + (r & 3) + 8 * (r >> 2);
          const double kv = gi + row_off == gid ? 1.0 : ex[q];
          if (colok && gi < n) dst[gi] = kv;
        }
      }
    }
    if (cstride <= 0) return;
    bn += cstride;
    __syncthreads();  // the next half rewrites the column tables the epilogue has just read
    continue;
  }
  if constexpr (GEMV) {
    // ---- GEMV epilogue: rowsum[r] = sum over this workgroup's 64 columns of coef * K (the same kernel
    // values as the stored path), lane-local over its two columns, then a 32-lane butterfly per row.
    const int64_t row0 = bm + w * 32 + 4 * h;
    double rs[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) rs[r] = 0.0;
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
      const int cl = bj * 32 + l32;
      const int64_t gj = bn + cl;
      const bool colok = gj < ncol;
      const double cf = colok ? coef[gj] : 0.0;
      const int64_t gid = colok ? int64_t(diag ? diag[gj] : colid[gj]) : -1;
      const int32_t nbj = n0_c[cl];
      const double wbj = EXTRA ? wn_c[cl] : 0.0;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        double ex[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int r = 8 * half + q;
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
          const int32_t D0 = n0_r[w * 32 + rl] + nbj - 2 * acc[bj][r];
          double dist = w0 * double(D0);
          if (EXTRA) dist += (wn_r[w * 32 + rl] + wbj) - 2.0 * xacc[bj][r];
          dist = dist > 0.0 ? dist : 0.0;
          ex[q] = neg_gamma * dist;
        }
        exp_batch<8>(ex);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int r = 8 * half + q;
          const int64_t gi = row0 + (r & 3) + 8 * (r >> 2);
          const double kv = gi + row_off == gid ? 1.0 : ex[q];
          rs[r] += cf * kv;  // columns outside the block carry cf = 0
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int off = 16; off > 0; off >>= 1) rs[r] += __shfl_xor(rs[r], off, 64);
    if (l32 == 0) {
      const int64_t part = (bn / QBN);  // this workgroup's 64-column half
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gi = row0 + (r & 3) + 8 * (r >> 2);
        if (gi < n) K[gi * ldk + part] = rs[r];
      }
    }
    if (cstride <= 0) return;
    bn += cstride;
    __syncthreads();  // the next half rewrites the column tables the epilogue has just read
    continue;
  }
  // ---- epilogue in the 32x32 accumulator layout: col = lane & 31,
  // row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5).
  double* im = img + w * (32 * 33);
  const bool mirror = !RECT && tm != tn;
  // Interior tiles (the vast majority) skip the per-element bounds tests; store addresses are a
  // per-lane base plus a wave-uniform (scalar) row offset.
  const bool interior = bm + QBM <= n && bn + QBM <= ncol;
  const int64_t row0 = bm + w * 32 + 4 * h;  // this lane's row for r = 0
#pragma unroll
  for (int bj = 0; bj < 2; ++bj) {
    const int cl = bj * 32 + l32;
    const int64_t gj = bn + cl;
    const int32_t nbj = n0_c[cl];
    const double wbj = EXTRA ? wn_c[cl] : 0.0;
    double* kp = K + row0 * ldk + gj;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      double ex[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = 8 * half + q;
        const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int32_t D0 = n0_r[w * 32 + rl] + nbj - 2 * acc[bj][r];  // exact
        double dist = w0 * double(D0);
        if (EXTRA) dist += (wn_r[w * 32 + rl] + wbj) - 2.0 * xacc[bj][r];
        dist = dist > 0.0 ? dist : 0.0;
        ex[q] = neg_gamma * dist;
      }
      exp_batch<8>(ex);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = 8 * half + q;
        const int ro = (r & 3) + 8 * (r >> 2);
        const int rl = ro + 4 * h;
        const int64_t gi = row0 + ro;
        const double kv = gi == c0 + gj ? 1.0 : ex[q];
        if (interior || (gi < n && gj < ncol)) __builtin_nontemporal_store(kv, kp + int64_t(ro) * ldk);
        if (mirror) im[l32 * 33 + rl] = kv;  // im[col][row]
      }
    }
    if (mirror) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // Mirrored rows = this tile's columns: 16 lanes per row, one 16-byte chunk each, so every
      // store instruction writes 4 whole 256-byte row segments.
      const int chunk = lane & 15;
      const int64_t gcol = bm + w * 32 + 2 * chunk;
      const int64_t mrow0 = bn + bj * 32 + (lane >> 4);
      double* mp = K + mrow0 * ldk + gcol;
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int mrow = it * 4 + (lane >> 4);
        const double* sp = im + mrow * 33 + 2 * chunk;
        double* dst = mp + int64_t(4 * it) * ldk;
        if (interior) {
          __builtin_nontemporal_store(f64x2{sp[0], sp[1]}, reinterpret_cast<f64x2*>(dst));
        } else if (mrow0 + 4 * it < n) {
          if (gcol + 1 < n)
            __builtin_nontemporal_store(f64x2{sp[0], sp[1]}, reinterpret_cast<f64x2*>(dst));
          else if (gcol < n)
            dst[0] = sp[0];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  return;
  }  // for (GEMV column halves)
}

// Narrow column store (decomposition column cache, <= kNarrowCols missing columns per f update): the
// columns are resident in LDS, 32 at a time, and every wave streams 32-row tiles of Q straight from
// HBM into its MFMA fragments, so an update that misses a handful of columns reads Q once at streaming
// rate instead of paying the 128 x 64 tiled pass.  The MFMA takes the COLUMNS as its A operand and the
// rows as B: the accumulator is K^T, lane l32 holds row l32 of the tile and register r column
// (r & 3) + 8 (r >> 2) + 4 h, so a store of register r writes two 256-byte runs of consecutive rows
// of two columns (the igram layout wrote 32 B pieces of 32 columns per store: 1.7 TB/s), the row
// norms are the lane's own, and whole quarters of registers whose columns lie beyond the group are
// skipped.  The integer products are exact and every (row, column) entry sees the same extra-group
// FP64 flushes in k-step order and the same epilogue arithmetic as igram_tri_kernel, so every stored
// value equals the GEMV's bit for bit.
constexpr int kNarrowCols = 64;
constexpr int kNarrowMaxKq = 1536;  // 32 x (kq + 16) bytes of columns in LDS
template <bool EXTRA>
__global__ __launch_bounds__(256, 3) void igram_colstore_narrow_kernel(
    const int8_t* __restrict__ Q, int64_t n, int kq, int main0, const int32_t* __restrict__ N0,
    const double* __restrict__ WN, const double* __restrict__ step_w, double w0, double neg_gamma,
    const int8_t* __restrict__ Qc, const int32_t* __restrict__ N0c, const double* __restrict__ WNc,
    const int32_t* __restrict__ ids, const int32_t* __restrict__ slots, const int32_t* __restrict__ count,
    int64_t row_off, double* __restrict__ cache, int64_t ldc, int kused, const int32_t* __restrict__ gate = nullptr,
    bool gsplit = false, bool all = false, const int32_t* __restrict__ diag = nullptr) {
  __shared__ double sw[kMaxSteps];
  __shared__ double wn_c[32];
  __shared__ int64_t off_c[32];
  __shared__ int32_t n0_c[32], id_c[32], dg_c[32];
  extern __shared__ __attribute__((aligned(16))) char nsm[];
  if (gate && *gate != 0) return;  // a stopped decomposition solve's remaining batch
  const int cnt = *count;
  // gsplit (a working set's K(W, W)): workgroup row blockIdx.y takes column group blockIdx.y only, any count
  // all: no tiled store was launched for this update, so every count is this kernel's (32 columns a pass)
  if (cnt <= 0 || (!gsplit && !all && cnt > kNarrowCols)) return;  // nothing missing, or the tiled store's
  const int LS = kq + 16;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, l32 = lane & 31, h = lane >> 5;
  const int main_step0 = main0 / 32;
  if (EXTRA)
    for (int k = t; k < main_step0; k += 256) sw[k] = step_w[k];
  const int64_t tiles = (n + 31) / 32;
  const int64_t wave0 = int64_t(blockIdx.x) * 4 + w, nwaves = int64_t(gridDim.x) * 4;
  const i32x4 zero4 = {0, 0, 0, 0};
  const i32x16 zero16 = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  // only the k-steps holding columns (kused: the trailing pad of kq is zero in every row, so its
  // MFMAs would add 0); a partial last chunk of 4 steps loads zeros for the steps beyond
  const int nsu = kused / 32, nch = (nsu + 3) / 4;  // nch * 4 <= kq / 32: kq is a multiple of 128
  for (int g0 = gsplit ? int(blockIdx.y) * 32 : 0; g0 < cnt; g0 += gsplit ? cnt : 32) {
    const int gc = min(32, cnt - g0);
    __syncthreads();  // the previous group's columns are consumed
    if (t < 32) {
      const bool ok = t < gc;
      const int32_t id = ok ? ids[g0 + t] : -1;
      id_c[t] = id;
      dg_c[t] = ok && diag ? diag[g0 + t] : id;
      off_c[t] = ok ? int64_t(slots[g0 + t]) * ldc : 0;
      n0_c[t] = ok ? N0c[id] : 0;
      if (EXTRA) wn_c[t] = ok ? WNc[id] : 0.0;
    }
    // the group's columns into LDS, eight 16-byte loads in flight per thread (one at a time, the 9
    // dependent round trips of a 1,152-byte column set were most of a K(W, W) workgroup's time)
    const int cpr = kq / 16;
    for (int c0 = 0; c0 < 32 * cpr; c0 += 256 * 8) {
      i32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = c0 + t + 256 * u, col = c / cpr, ch = c - col * cpr;
        v[u] = c < 32 * cpr && col < gc ? *reinterpret_cast<const i32x4*>(Qc + int64_t(ids[g0 + col]) * kq + ch * 16)
                                        : zero4;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = c0 + t + 256 * u, col = c / cpr, ch = c - col * cpr;
        if (c < 32 * cpr) *reinterpret_cast<i32x4*>(nsm + col * LS + ch * 16) = v[u];
      }
    }
    __syncthreads();
    const char* bcol = nsm + l32 * LS + 16 * h;  // column l32's fragment (the A operand)
    // the wave's (tile, chunk of 4 k-steps) positions as one stream, loads one chunk ahead (across tile
    // boundaries: the next tile's first chunk is in flight during this tile's epilogue; two ahead
    // measured the same)
    int64_t lt = wave0;
    int lc = 0;
    auto ld = [&](i32x4(&dst)[4]) {
      const int64_t arow = lt * 32 + l32;
      const bool ok = lt < tiles && arow < n;
      const int8_t* ap = Q + (ok ? arow : 0) * int64_t(kq) + 16 * h + lc * 128;
#pragma unroll
      for (int u = 0; u < 4; ++u) dst[u] = ok && 4 * lc + u < nsu ? *reinterpret_cast<const i32x4*>(ap + u * 32) : zero4;
      if (++lc == nch) {
        lc = 0;
        lt += nwaves;
      }
    };
    i32x4 p0[4];
    ld(p0);
    for (int64_t tile = wave0; tile < tiles; tile += nwaves) {
      // the lane's row norms, loaded now so their latency hides behind the k-loop
      const int64_t gi = tile * 32 + l32;
      const bool rowok = gi < n;
      const int32_t n0_row = N0[rowok ? gi : 0];
      const double wn_row = EXTRA ? WN[rowok ? gi : 0] : 0.0;
      i32x16 acc = zero16;
      double xacc[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) xacc[r] = 0.0;
      bool fresh = false;
      for (int c = 0; c < nch; ++c) {
        i32x4 cur[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) cur[u] = p0[u];
        ld(p0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int step = 4 * c + u;
          const i32x4 b = *reinterpret_cast<const i32x4*>(bcol + step * 32);
          if (EXTRA && fresh) {
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, cur[u], zero16, 0, 0, 0);
            fresh = false;
          } else {
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, cur[u], acc, 0, 0, 0);
          }
          if (EXTRA && step < main_step0) {
            const double wgt = sw[step];
            if (wgt != 0.0) {  // last k-step of an extra group: flush its exact cross term
#pragma unroll
              for (int r = 0; r < 16; ++r)
                if (2 * (r & ~3) < gc) xacc[r] = __builtin_fma(wgt, double(acc[r]), xacc[r]);  // quarters of real columns only
              fresh = true;
            }
          }
        }
      }
#pragma unroll
      for (int qtr = 0; qtr < 4; ++qtr) {  // registers 4 qtr .. 4 qtr + 3: columns 8 qtr + 4 h + (0..3)
        if (8 * qtr >= gc) break;
        double ex[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 4 * qtr + q, cc = q + 8 * qtr + 4 * h;
          const int32_t D0 = n0_row + n0_c[cc] - 2 * acc[r];
          double dist = w0 * double(D0);
          if (EXTRA) dist += (wn_row + wn_c[cc]) - 2.0 * xacc[r];
          dist = dist > 0.0 ? dist : 0.0;
          ex[q] = neg_gamma * dist;
        }
        exp_batch<4>(ex);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cc = q + 8 * qtr + 4 * h;
          const double kv = gi + row_off == int64_t(dg_c[cc]) ? 1.0 : ex[q];
          if (cc < gc && rowok) cache[off_c[cc] + gi] = kv;
        }
      }
    }
  }
}

}  // namespace

int exp_selftest(hipStream_t s, const double* x, int64_t n, double* out_lib, double* out_batch) {
  if (n <= 0) return SVM_OK;
  hipLaunchKernelGGL(exp_check_kernel, dim3(unsigned((n + 2047) / 2048)), dim3(256), 0, s, x, n, out_lib, out_batch);
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

// Host-side column plan (from the training min/max): the main group (most common range) and the
// extra groups, each padded to a 32-column k-step, with per-column centring offsets.
bool plan_quant(const double* mn, const double* mx, int64_t d, QuantPlan* P) {
  P->ok = false;
  if (!mn || !mx || d <= 0) return false;
  std::map<double, std::vector<int32_t>> by_range;  // range -> columns
  for (int64_t j = 0; j < d; ++j) {
    const double rng = mx[j] - mn[j];
    if (!(rng >= 1e-12)) continue;  // constant column: scaled to 0 everywhere, contributes nothing
    if (rng > 255.0 + 1e-9 || rng != std::floor(rng)) return false;  // integer data has integer ranges
    by_range[rng].push_back(int32_t(j));
  }
  if (by_range.empty()) return false;
  // Exact group merging: a column of range r joins a group of range R when r divides R -- its
  // integers q in [0, r] become q * R / r in [0, R], and (dq)^2 / r^2 = (dq * R / r)^2 / R^2 -- so pixel
  // columns whose maxima divide 255 (1, 3, 5, 15, 17, 51, 85) join the main group, and small ranges
  // join any larger group they divide, each merge saving a padded k-step and an FP64 flush per tile.
  // Ranges are placed from the most populated down; the first group each one divides takes it.
  std::vector<std::pair<double, size_t>> order;
  for (const auto& kv : by_range) order.emplace_back(kv.first, kv.second.size());
  std::stable_sort(order.begin(), order.end(), [](const auto& a, const auto& b) {
    return a.second != b.second ? a.second > b.second : a.first > b.first;
  });
  std::vector<double> targets;                    // group ranges in creation order
  std::map<double, std::vector<int32_t>> groups;  // group range -> columns
  std::vector<double> r(static_cast<size_t>(d), 0.0);  // per column: its group's range
  for (const auto& [rng, cnt] : order) {
    double to = rng;
    for (double T : targets)
      if (std::fmod(T, rng) == 0.0) {
        to = T;
        break;
      }
    if (to == rng) targets.push_back(rng);
    for (int32_t j : by_range[rng]) {
      r[size_t(j)] = to;
      groups[to].push_back(j);
    }
  }
  for (auto& kv : groups) std::sort(kv.second.begin(), kv.second.end());
  const std::vector<int32_t>* main = nullptr;
  double rmain = 0.0;
  for (const auto& kv : groups)
    if (!main || kv.second.size() > main->size()) {
      main = &kv.second;
      rmain = kv.first;
    }
  P->w0 = 1.0 / (rmain * rmain);
  P->perm.clear();
  P->step_w.clear();
  auto pad_to = [&](size_t m) {
    while (P->perm.size() % m) P->perm.push_back(-1);
  };
  for (const auto& kv : groups) {
    if (kv.first == rmain) continue;
    const double wg = 1.0 / (kv.first * kv.first);
    for (int32_t j : kv.second) P->perm.push_back(j);
    pad_to(32);
    const size_t steps = P->perm.size() / 32;
    P->step_w.resize(steps, 0.0);
    P->step_w[steps - 1] = wg;  // flush at the group's last k-step
  }
  P->main0 = int(P->perm.size());
  for (int32_t j : *main) P->perm.push_back(j);
  pad_to(kColAlign);
  P->kq = int(P->perm.size());
  if (P->kq / 32 > kMaxSteps) return false;
  P->rmul.assign(P->perm.size(), 0.0);
  P->off.assign(P->perm.size(), 0.0);
  P->wx.assign(P->perm.size(), 0.0);
  for (size_t k = 0; k < P->perm.size(); ++k) {
    const int32_t j = P->perm[k];
    if (j < 0) continue;
    const double rj = r[size_t(j)];
    P->rmul[k] = rj;
    P->off[k] = std::ceil(rj * 0.5);  // q - ceil(r/2) in [-128, 127] for r <= 255
    if (int(k) < P->main0) P->wx[k] = 1.0 / (rj * rj);
  }
  if (P->step_w.empty()) P->step_w.push_back(0.0);
  P->n_groups = int(groups.size());
  P->ok = true;
  return true;
}


// Quantise n (scaled) rows into Q (n x P.kq int8), N0, WN.  *ok = false when some value is not an
// integer multiple of 1/r_j in [0, 255/r_j] (nothing usable written).  aux: device scratch of
// quantize_aux_bytes(P) bytes for the column tables.  Synchronises the stream (reads the flag).
size_t quantize_aux_bytes(const QuantPlan& P) {
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  return al(P.perm.size() * 4) + 3 * al(P.perm.size() * 8) + 256;
}

int quantize_rows(hipStream_t s, const double* X, int64_t n, int64_t ld, const QuantPlan& P, void* aux, int8_t* Q,
                  int32_t* N0, double* WN, bool* ok) {
  *ok = false;
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  char* p = static_cast<char*>(aux);
  auto take = [&](size_t bytes) {
    char* q = p;
    p += al(bytes);
    return q;
  };
  auto* perm = reinterpret_cast<int32_t*>(take(P.perm.size() * 4));
  auto* rmul = reinterpret_cast<double*>(take(P.rmul.size() * 8));
  auto* off = reinterpret_cast<double*>(take(P.off.size() * 8));
  auto* wx = reinterpret_cast<double*>(take(P.wx.size() * 8));
  auto* fail = reinterpret_cast<unsigned*>(take(4));
  SVMD_CHECK(hipMemcpyAsync(perm, P.perm.data(), P.perm.size() * 4, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(rmul, P.rmul.data(), P.rmul.size() * 8, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(off, P.off.data(), P.off.size() * 8, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(wx, P.wx.data(), P.wx.size() * 8, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemsetAsync(fail, 0, 4, s));
  if (n > 0 && P.kq <= kQuantLdsMaxKq) {
    const size_t lds = size_t(P.kq) * 8 + size_t(P.main0) * 8;
    const unsigned blocks = unsigned(std::min<int64_t>((n + 3) / 4, 2048));
    hipLaunchKernelGGL(quantize_rows_lds_kernel, dim3(blocks), dim3(256), lds, s, X, n, ld, perm, rmul, off, wx,
                       P.main0, P.kq, Q, N0, WN, fail);
    SVMD_LAUNCH_CHECK();
  } else if (n > 0) {
    hipLaunchKernelGGL(quantize_rows_kernel, dim3(unsigned((n + 3) / 4)), dim3(256), 0, s, X, n, ld, perm, rmul, off,
                       wx, P.main0, P.kq, Q, N0, WN, fail);
    SVMD_LAUNCH_CHECK();
  }
  unsigned hfail = 1;
  SVMD_CHECK(hipMemcpyAsync(&hfail, fail, 4, hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipStreamSynchronize(s));
  *ok = hfail == 0;
  return SVM_OK;
}

size_t igram_workspace(int64_t n, const QuantPlan& P) {
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  return al(size_t(n) * size_t(P.kq)) + al(size_t(n) * 4) + al(size_t(n) * 8) + al(P.step_w.size() * 8) +
         quantize_aux_bytes(P);
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
  auto take = [&](size_t bytes) {
    char* q = p;
    p += al(bytes);
    return q;
  };
  auto* Q = reinterpret_cast<int8_t*>(take(size_t(n) * size_t(P.kq)));
  auto* N0 = reinterpret_cast<int32_t*>(take(size_t(n) * 4));
  auto* WN = reinterpret_cast<double*>(take(size_t(n) * 8));
  auto* stw = reinterpret_cast<double*>(take(P.step_w.size() * 8));
  bool ok = false;
  int rc = quantize_rows(s, X, n, ld, P, p, Q, N0, WN, &ok);
  if (rc) return rc;
  if (!ok) return SVM_OK;  // not integer-valued: caller uses the FP64 path
  rc = launch_igram_sym(s, Q, N0, WN, stw, n, P, gamma, K, ldk);
  if (rc) return rc;
  *used = true;
  return SVM_OK;
}

// The symmetric exact-integer Gram of quantised rows (Q, N0, WN); stw: device scratch for the step
// weights.
int launch_igram_sym(hipStream_t s, const int8_t* Q, const int32_t* N0, const double* WN, double* stw, int64_t n,
                     const QuantPlan& P, double gamma, double* K, int64_t ldk, bool copy_stw, const int32_t* gate) {
  if (copy_stw) SVMD_CHECK(hipMemcpyAsync(stw, P.step_w.data(), P.step_w.size() * 8, hipMemcpyHostToDevice, s));
  const int64_t tiles = (n + QBM - 1) / QBM;
  const int64_t nwg = tiles * (tiles + 1);  // two 128x64 halves per upper-triangular 128x128 tile
  if (nwg > 0x7FFFFFFF) {
    set_error("igram: problem too large for one launch");
    return SVM_ERR_ARG;
  }
  int bk = P.kq % 128 == 0 ? 128 : 64;  // fewer, deeper stages when the column count allows
  if (const char* v = getenv("SVM355_IGRAM_BK")) bk = atoi(v) == 64 || P.kq % 128 ? 64 : 128;
#define SVM_IGRAM(EX, B)                                                                                    \
  hipLaunchKernelGGL((igram_tri_kernel<EX, B>), dim3(unsigned(nwg)), dim3(256), 0, s, Q, n, P.kq, P.main0, N0, \
                     WN, stw, P.w0, -gamma, K, ldk, tiles, int64_t(0), int64_t(0), nullptr, nullptr, nullptr, nullptr, \
                     nullptr, nullptr, int64_t(0), gate)
  if (P.main0 > 0) {
    if (bk == 128) SVM_IGRAM(true, 128); else SVM_IGRAM(true, 64);
  } else {
    if (bk == 128) SVM_IGRAM(false, 128); else SVM_IGRAM(false, 64);
  }
#undef SVM_IGRAM
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

// Quantise uint8 pixel rows Xu (n x d, contiguous, device) straight from the bytes with the plan P
// built from their column min / max (host, d values): Q (n x P.kq), N0, WN exactly as
// quantize_rows on the scaled FP64 rows.  *ok = false (nothing usable) when the plan does not apply
// to these statistics (non-integer minima or ranges) or a value fails the check.  aux holds
// quantize_u8_aux_bytes(P) bytes.  Synchronises the stream (reads the flag).
size_t quantize_u8_aux_bytes(const QuantPlan& P) {
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  return 2 * al(P.perm.size() * 4) + al(P.wx.size() * 8) + 256;
}

int quantize_u8_rows(hipStream_t s, const uint8_t* Xu, int64_t n, int64_t d, const double* mn_h, const double* mx_h,
                     const QuantPlan& P, void* aux, int8_t* Q, int32_t* N0, double* WN, bool* ok) {
  *ok = false;
  if (!P.ok || n <= 0 || P.kq > kQuantLdsMaxKq) return SVM_OK;
  std::vector<int32_t> pack(P.perm.size(), 0);
  for (size_t k = 0; k < P.perm.size(); ++k) {
    const int32_t j = P.perm[k];
    if (j < 0) continue;
    const double mn = mn_h[j], rj = mx_h[j] - mn_h[j], fac = P.rmul[k] / rj;
    if (mn != std::floor(mn) || mn < 0 || mn > 255 || fac != std::floor(fac) || fac < 1 || fac > 255 ||
        P.off[k] > 255)
      return SVM_OK;
    pack[k] = int32_t(mn) | (int32_t(fac) << 8) | (int32_t(P.off[k]) << 16);
  }
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  char* p = static_cast<char*>(aux);
  auto take = [&](size_t bytes) {
    char* q = p;
    p += al(bytes);
    return q;
  };
  auto* perm = reinterpret_cast<int32_t*>(take(P.perm.size() * 4));
  auto* pk = reinterpret_cast<int32_t*>(take(P.perm.size() * 4));
  auto* wx = reinterpret_cast<double*>(take(P.wx.size() * 8));
  auto* fail = reinterpret_cast<unsigned*>(take(4));
  SVMD_CHECK(hipMemcpyAsync(perm, P.perm.data(), P.perm.size() * 4, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(pk, pack.data(), pack.size() * 4, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemcpyAsync(wx, P.wx.data(), P.wx.size() * 8, hipMemcpyHostToDevice, s));
  SVMD_CHECK(hipMemsetAsync(fail, 0, 4, s));
  const size_t lds = size_t(P.kq) * 8 + size_t(P.main0) * 8;
  const unsigned blocks = unsigned(std::min<int64_t>((n + 3) / 4, 2048));
  hipLaunchKernelGGL(quantize_u8_lds_kernel, dim3(blocks), dim3(256), lds, s, Xu, n, d, perm, pk, wx, P.main0, P.kq,
                     Q, N0, WN, fail);
  SVMD_LAUNCH_CHECK();
  unsigned hfail = 1;
  SVMD_CHECK(hipMemcpyAsync(&hfail, fail, 4, hipMemcpyDeviceToHost, s));
  SVMD_CHECK(hipStreamSynchronize(s));
  *ok = hfail == 0;
  return SVM_OK;
}

// run_igram on uint8 pixel rows Xu (n x d, contiguous, device) whose column min / max (host, d
// values) the plan was built from: quantised without FP64 rows.  *used = false (nothing written)
// when the plan does not apply to these statistics (non-integer minima or ranges).
int run_igram_u8(hipStream_t s, const uint8_t* Xu, int64_t n, int64_t d, const double* mn_h, const double* mx_h,
                 const QuantPlan& P, double gamma, double* K, int64_t ldk, void* ws, bool* used) {
  *used = false;
  if (!P.ok || n <= 0 || P.kq > kQuantLdsMaxKq) return SVM_OK;
  if (ldk < n) {
    set_error("igram: ldk < n");
    return SVM_ERR_ARG;
  }
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  char* p = static_cast<char*>(ws);
  auto take = [&](size_t bytes) {
    char* q = p;
    p += al(bytes);
    return q;
  };
  auto* Q = reinterpret_cast<int8_t*>(take(size_t(n) * size_t(P.kq)));
  auto* N0 = reinterpret_cast<int32_t*>(take(size_t(n) * 4));
  auto* WN = reinterpret_cast<double*>(take(size_t(n) * 8));
  auto* stw = reinterpret_cast<double*>(take(P.step_w.size() * 8));
  bool ok = false;
  int rc = quantize_u8_rows(s, Xu, n, d, mn_h, mx_h, P, p, Q, N0, WN, &ok);
  if (rc) return rc;
  if (!ok) return SVM_OK;
  rc = launch_igram_sym(s, Q, N0, WN, stw, n, P, gamma, K, ldk);
  if (rc) return rc;
  *used = true;
  return SVM_OK;
}

size_t igram_u8_workspace(int64_t n, const QuantPlan& P) {
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  return al(size_t(n) * size_t(P.kq)) + al(size_t(n) * 4) + al(size_t(n) * 8) + al(P.step_w.size() * 8) +
         2 * al(P.perm.size() * 4) + al(P.wx.size() * 8) + 256;
}

// K(rows [0, n), rows [0, ncols)) of the same (scaled) rows on the exact-integer path, ncols <= n,
// into K (n x ldk, ldk >= ncols): bit-identical to those entries of run_igram's Gram.  ws holds
// igram_workspace(n, P) bytes; *used = false (nothing written) when the data are not integer-valued.
int run_igram_block(hipStream_t s, const double* X, int64_t n, int64_t ld, int64_t ncols, const QuantPlan& P,
                    double gamma, double* K, int64_t ldk, void* ws, bool* used) {
  *used = false;
  if (!P.ok || n <= 0 || ncols <= 0) return SVM_OK;
  if (ncols > n || ldk < ncols) {
    set_error("igram block: need ncols <= n and ldk >= ncols");
    return SVM_ERR_ARG;
  }
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  char* p = static_cast<char*>(ws);
  auto take = [&](size_t bytes) {
    char* q = p;
    p += al(bytes);
    return q;
  };
  auto* Q = reinterpret_cast<int8_t*>(take(size_t(n) * size_t(P.kq)));
  auto* N0 = reinterpret_cast<int32_t*>(take(size_t(n) * 4));
  auto* WN = reinterpret_cast<double*>(take(size_t(n) * 8));
  auto* stw = reinterpret_cast<double*>(take(P.step_w.size() * 8));
  bool ok = false;
  int rc = quantize_rows(s, X, n, ld, P, p, Q, N0, WN, &ok);
  if (rc) return rc;
  if (!ok) return SVM_OK;
  SVMD_CHECK(hipMemcpyAsync(stw, P.step_w.data(), P.step_w.size() * 8, hipMemcpyHostToDevice, s));
  const int64_t tiles = (n + QBM - 1) / QBM, ctiles = (ncols + QBM - 1) / QBM;
  const int64_t nwg = 2 * tiles * ctiles;  // two 128x64 halves per tile
  if (nwg > 0x7FFFFFFF) {
    set_error("igram block: problem too large for one launch");
    return SVM_ERR_ARG;
  }
  const int bk = P.kq % 128 == 0 ? 128 : 64;
#define SVM_IGRAM_BLOCK(EX, B)                                                                                 \
  hipLaunchKernelGGL((igram_tri_kernel<EX, B, true>), dim3(unsigned(nwg)), dim3(256), 0, s, Q, n, P.kq, P.main0, \
                     N0, WN, stw, P.w0, -gamma, K, ldk, tiles, ncols)
  if (P.main0 > 0) {
    if (bk == 128) SVM_IGRAM_BLOCK(true, 128); else SVM_IGRAM_BLOCK(true, 64);
  } else {
    if (bk == 128) SVM_IGRAM_BLOCK(false, 128); else SVM_IGRAM_BLOCK(false, 64);
  }
#undef SVM_IGRAM_BLOCK
  SVMD_LAUNCH_CHECK();
  *used = true;
  return SVM_OK;
}

// Decomposition solver f update (decomp.hip): part[i * ldp + c] = sum over the c-th 64-column half of
// coef[k] * K(i, cols[k]) for every row i < n of (Q, N0, WN) -- global row row_off + i of the full
// quantised set (Qc, N0c, WNc) the column ids index -- and k < *mcount (device; <= m, the grid's
// bound).  ldp >= 2 * ceil(m / 128); halves at or beyond *mcount are not written: the caller sums
// the first ceil(*mcount / 64) in index order.
int launch_igram_gemv(hipStream_t s, const int8_t* Q, const int32_t* N0, const double* WN, const double* stw,
                      int64_t n, int64_t row_off, const int8_t* Qc, const int32_t* N0c, const double* WNc,
                      const int32_t* cols, const double* coef, const int32_t* mcount, int64_t m, const QuantPlan& P,
                      double gamma, double* part, int64_t ldp, const int32_t* diag) {
  if (n <= 0 || m <= 0) return SVM_OK;
  const int64_t tiles = (n + QBM - 1) / QBM, ctiles = (m + QBM - 1) / QBM;
  // the grid covers gc 128-column tiles per row tile; its workgroups walk further halves when *mcount
  // exceeds them (SVM355_GEMV_GC; 0 = one workgroup per half of all m columns, most exiting at once;
  // -1 = one workgroup per row tile walking every half).  Measured (per call at 60k / 250k fit): gc 0
  // 113 us / 137 ms, gc 1 90 us / 109 ms, -1 82 us / 98 ms
  // (profiles/r3_decomp_gemv_grid_ab.txt)
  // Walking needs enough row tiles to fill the chip: below 256 (fewer than 32k rows, e.g. one GPU's
  // share in the distributed solve) one workgroup per half keeps every half of every tile in flight.
  int64_t gc = tiles >= 256 ? -1 : 0;
  if (const char* v = getenv("SVM355_GEMV_GC")) gc = atoi(v);
  const bool walk_all = gc < 0;  // -1: one workgroup per row tile walking every 64-column half
  if (!walk_all && (gc == 0 || gc > ctiles)) gc = ctiles;
  const int64_t cstride = walk_all ? QBN : gc < ctiles ? gc * QBM : 0;
  if (walk_all) gc = 1;
  const int64_t nwg = walk_all ? tiles : 2 * tiles * gc;
  if (ldp < 2 * ctiles || nwg > 0x7FFFFFFF) {
    set_error("igram gemv: bad partial stride or problem too large");
    return SVM_ERR_ARG;
  }
  int bk = P.kq % 128 == 0 ? 128 : 64;
  if (const char* v = getenv("SVM355_GEMV_BK")) bk = atoi(v) == 64 || P.kq % 128 ? 64 : 128;  // A/B knob
#define SVM_IGRAM_GEMV(EX, B)                                                                                       \
  hipLaunchKernelGGL((igram_tri_kernel<EX, B, true, true>), dim3(unsigned(nwg)), dim3(256), 0, s, Q, n, P.kq,        \
                     P.main0, N0, WN, stw, P.w0, -gamma, part, ldp, tiles, gc * QBM, int64_t(0), cols, coef, mcount, Qc,  \
                     N0c, WNc, row_off, nullptr, cstride, nullptr, diag)
  if (P.main0 > 0) {
    if (bk == 128) SVM_IGRAM_GEMV(true, 128); else SVM_IGRAM_GEMV(true, 64);
  } else {
    if (bk == 128) SVM_IGRAM_GEMV(false, 128); else SVM_IGRAM_GEMV(false, 64);
  }
#undef SVM_IGRAM_GEMV
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

// Decomposition column cache (decomp.hip): cache[slots[k] * ldc + i] = K(row_off + i, ids[k]) for the
// rows i < n of (Q, N0, WN) and k < *count (device; <= m, the grid's bound) -- the GEMV's operands,
// grid and kernel values (bit for bit), stored per column instead of reduced.
int launch_igram_colstore(hipStream_t s, const int8_t* Q, const int32_t* N0, const double* WN, const double* stw,
                          int64_t n, int64_t row_off, const int8_t* Qc, const int32_t* N0c, const double* WNc,
                          const int32_t* ids, const int32_t* slots, const int32_t* count, int64_t m,
                          const QuantPlan& P, double gamma, double* cache, int64_t ldc, const int32_t* gate,
                          bool tiled, const int32_t* diag) {
  if (n <= 0 || m <= 0) return SVM_OK;
  const bool narrow_all = !tiled && gate && P.kq <= kNarrowMaxKq;  // the narrow store alone, any count
  if (gate && P.kq <= kNarrowMaxKq) {  // <= kNarrowCols columns: the streaming kernel (the tiled one exits)
    const int64_t tiles = (n + 31) / 32;
    const size_t lds = size_t(32) * (P.kq + 16);
    int kused = 0;  // int8 columns up to the last real one, rounded up to a k-step
    for (int k = int(P.perm.size()) - 1; k >= 0; --k)
      if (P.perm[k] >= 0) {
        kused = k + 1;
        break;
      }
    kused = std::min(P.kq, (std::max(kused, 1) + 31) / 32 * 32);
    // one resident wave of workgroups (each loads its columns once and walks ~tiles / waves tiles): a
    // 2048-workgroup grid ran 2.7 rounds at 3 workgroups per CU
    int dev = 0, cus = 256, per_cu = 3;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (P.main0 > 0)
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, igram_colstore_narrow_kernel<true>, 256, lds);
    else
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, igram_colstore_narrow_kernel<false>, 256, lds);
    if (const char* v = getenv("SVM355_NARROW_WGS_PER_CU")) per_cu = std::max(1, atoi(v));  // A/B: grid size
    const unsigned nwg = unsigned(std::max<int64_t>(1, std::min<int64_t>((tiles + 3) / 4, int64_t(cus) * std::max(per_cu, 1))));
    if (P.main0 > 0)
      hipLaunchKernelGGL(igram_colstore_narrow_kernel<true>, dim3(nwg), dim3(256), lds, s, Q, n, P.kq, P.main0, N0,
                         WN, stw, P.w0, -gamma, Qc, N0c, WNc, ids, slots, count, row_off, cache, ldc, kused, nullptr,
                         false, narrow_all, diag);
    else
      hipLaunchKernelGGL(igram_colstore_narrow_kernel<false>, dim3(nwg), dim3(256), lds, s, Q, n, P.kq, P.main0, N0,
                         WN, stw, P.w0, -gamma, Qc, N0c, WNc, ids, slots, count, row_off, cache, ldc, kused, nullptr,
                         false, narrow_all, diag);
    SVMD_LAUNCH_CHECK();
    if (narrow_all) return SVM_OK;
  }
  const int64_t tiles = (n + QBM - 1) / QBM, ctiles = (m + QBM - 1) / QBM;
  int64_t gc = tiles >= 256 ? -1 : 0;  // the GEMV's grid rule (launch_igram_gemv)
  if (const char* v = getenv("SVM355_GEMV_GC")) gc = atoi(v);
  const bool walk_all = gc < 0;
  if (!walk_all && (gc == 0 || gc > ctiles)) gc = ctiles;
  const int64_t cstride = walk_all ? QBN : gc < ctiles ? gc * QBM : 0;
  if (walk_all) gc = 1;
  const int64_t nwg = walk_all ? tiles : 2 * tiles * gc;
  if (ldc < n || nwg > 0x7FFFFFFF) {
    set_error("igram colstore: bad slot stride or problem too large");
    return SVM_ERR_ARG;
  }
  const int bk = P.kq % 128 == 0 ? 128 : 64;
#define SVM_IGRAM_CST(EX, B)                                                                                        \
  hipLaunchKernelGGL((igram_tri_kernel<EX, B, true, true, true>), dim3(unsigned(nwg)), dim3(256), 0, s, Q, n, P.kq,  \
                     P.main0, N0, WN, stw, P.w0, -gamma, cache, ldc, tiles, gc * QBM, int64_t(0), ids, nullptr, count,  \
                     Qc, N0c, WNc, row_off, P.kq <= kNarrowMaxKq ? gate : nullptr, cstride, slots, diag)
  if (P.main0 > 0) {
    if (bk == 128) SVM_IGRAM_CST(true, 128); else SVM_IGRAM_CST(true, 64);
  } else {
    if (bk == 128) SVM_IGRAM_CST(false, 128); else SVM_IGRAM_CST(false, 64);
  }
#undef SVM_IGRAM_CST
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

// K(W, W) of a decomposition working set (decomp.hip): the gathered quantised rows (Qw, N0w, WNw; n of
// them, rows beyond the set's size are stale but valid) against themselves through the narrow column
// store -- column group g of 32 in workgroup row g, row tiles over the workgroup columns: 32 x 8
// workgroups for 1,024 rows where the triangular Gram launch has 72, and the same kernel values bit
// for bit.  ids: the identity 0 .. n-1 on the device (columns k at K + k * ldk; K(W, W) is symmetric,
// so that is also its row k); the diagonal is 1 (local row == column).  false when kq is too wide.
int launch_igram_ww(hipStream_t s, const int8_t* Qw, const int32_t* N0w, const double* WNw, const double* stw,
                    int64_t n, const int32_t* ids, const int32_t* count, const QuantPlan& P, double gamma, double* K,
                    int64_t ldk, const int32_t* gate, bool* launched) {
  *launched = false;
  if (P.kq > kNarrowMaxKq || n <= 0 || n > 32 * 65535) return SVM_OK;  // not applicable: the caller's fallback
  int kused = 0;
  for (int k = int(P.perm.size()) - 1; k >= 0; --k)
    if (P.perm[k] >= 0) {
      kused = k + 1;
      break;
    }
  kused = std::min(P.kq, (std::max(kused, 1) + 31) / 32 * 32);
  const size_t lds = size_t(32) * (P.kq + 16);
  const dim3 grid(unsigned((n + 127) / 128), unsigned((n + 31) / 32));
  if (P.main0 > 0)
    hipLaunchKernelGGL(igram_colstore_narrow_kernel<true>, grid, dim3(256), lds, s, Qw, n, P.kq, P.main0, N0w, WNw, stw,
                       P.w0, -gamma, Qw, N0w, WNw, ids, ids, count, int64_t(0), K, ldk, kused, gate, true);
  else
    hipLaunchKernelGGL(igram_colstore_narrow_kernel<false>, grid, dim3(256), lds, s, Qw, n, P.kq, P.main0, N0w, WNw,
                       stw, P.w0, -gamma, Qw, N0w, WNw, ids, ids, count, int64_t(0), K, ldk, kused, gate, true);
  SVMD_LAUNCH_CHECK();  // a launch error (or one an earlier kernel left) is reported, never a silent fallback
  *launched = true;
  return SVM_OK;
}

// K(rows [0, n), rows [col0, col0 + ncols)) of already quantised rows (Q, N0, WN; step weights
// on the device in stw) into K (n x ldk, ldk >= ncols): a distributed-SMO team's slab, bit-identical
// to those entries of the symmetric Gram.
int launch_igram_slab(hipStream_t s, const int8_t* Q, const int32_t* N0, const double* WN, const double* stw,
                      int64_t n, int64_t col0, int64_t ncols, const QuantPlan& P, double gamma, double* K,
                      int64_t ldk) {
  if (n <= 0 || ncols <= 0) return SVM_OK;
  if (col0 < 0 || col0 + ncols > n || ldk < ncols) {
    set_error("igram slab: need 0 <= col0, col0 + ncols <= n and ldk >= ncols");
    return SVM_ERR_ARG;
  }
  const int64_t tiles = (n + QBM - 1) / QBM, ctiles = (ncols + QBM - 1) / QBM;
  const int64_t nwg = 2 * tiles * ctiles;
  if (nwg > 0x7FFFFFFF) {
    set_error("igram slab: problem too large for one launch");
    return SVM_ERR_ARG;
  }
  const int bk = P.kq % 128 == 0 ? 128 : 64;
#define SVM_IGRAM_SLAB(EX, B)                                                                                  \
  hipLaunchKernelGGL((igram_tri_kernel<EX, B, true>), dim3(unsigned(nwg)), dim3(256), 0, s, Q, n, P.kq, P.main0, \
                     N0, WN, stw, P.w0, -gamma, K, ldk, tiles, ncols, col0)
  if (P.main0 > 0) {
    if (bk == 128) SVM_IGRAM_SLAB(true, 128); else SVM_IGRAM_SLAB(true, 64);
  } else {
    if (bk == 128) SVM_IGRAM_SLAB(false, 128); else SVM_IGRAM_SLAB(false, 64);
  }
#undef SVM_IGRAM_SLAB
  SVMD_LAUNCH_CHECK();
  return SVM_OK;
}

}  // namespace svm355

SVMD_TU_WARM(igram)
