// Persistent SMO solver core (device code shared by smo.hip and dsmo.hip): the solver state block,
// the wave64 arg-reductions, the row sources (resident Gram, HBM row cache, distributed K(:, own)
// slab) and persist_solve, the whole SMO in one launch of co-resident workgroups exchanging tagged
// granules.  Everything is in an anonymous namespace: each translation unit instantiates its own
// kernels from it.
#pragma once
#include <cstdint>

#include "ctx.h"
#include "dsmo.h"
#include "qrows.h"

namespace svm355 {
namespace {

struct SmoState {
  int64_t ih, il;       // pair updated by the last step (consumed by the next select)
  double ch, cl;        // f-update coefficients (alpha_new - alpha) * y for ih / il
  double b_high, b_low;
  int64_t num_iter;     // reference counter (starts at 1)
  int32_t pending;      // 1 -> (ih, il, ch, cl) not yet applied to f
  int32_t stop;         // enum svm_stop
};

// ------------------------------------------------------------------------------------------------
// Persistent SMO: the whole solve in ONE launch.
//
// G workgroups (G <= #CUs, all co-resident) each own a contiguous slice of the training points and
// keep f, alpha and y of that slice in registers for the entire solve.  One iteration:
//   1. local masked argmin over I_high / argmax over I_low of the slice (wave64 butterfly + LDS),
//      carrying alpha of the winners;
//   2. publish the workgroup's two candidates as ten 8-byte {epoch, 32-bit payload} granules with
//      agent-scope relaxed (sc1) stores — a granule is written by one store and needs no fence;
//   3. wave 0 of EVERY workgroup sweeps all G candidate records (relaxed agent loads, s_sleep
//      between polls) until every tag equals the epoch, and reduces them with the lowest-index
//      rule: every workgroup obtains the identical (i_high, i_low, b_high, b_low, alpha_h, alpha_l);
//   4. every workgroup evaluates the stop tests and the two-variable update redundantly (same
//      inputs, same instruction sequence -> same bits), issuing the K11/K22/K12 and y loads in the
//      same memory round trip as its slice of rows K[i_high,:] and K[i_low,:];
//   5. the owners of i_high / i_low update their register alpha; every slice applies the f update.
// Records are double-buffered by epoch parity (a workgroup can be at most one epoch ahead of the
// slowest reader).  Every spin is bounded; a timeout sets *err and all workgroups drain.
// Per iteration this costs one HBM round trip plus one all-to-all granule exchange, instead of two
// kernel boundaries and a single-workgroup tail (smo_select_kernel + smo_step_kernel).
constexpr int kGranules = 10;    // per candidate record
constexpr int kRecStride = 16;   // granules per record slot (128 B)
constexpr int kMaxG = 64;        // one sweep pass: lane L of wave 0 reads workgroup L's record
constexpr uint32_t kSentinel = 0x7FFFFFFFu;  // "no candidate" index (n < 2^31)

__device__ __forceinline__ uint32_t lo32(double x) { return uint32_t(__double_as_longlong(x)); }
__device__ __forceinline__ uint32_t hi32(double x) { return uint32_t(uint64_t(__double_as_longlong(x)) >> 32); }
__device__ __forceinline__ double mk64(uint32_t lo, uint32_t hi) {
  return __longlong_as_double(int64_t((uint64_t(hi) << 32) | lo));
}

// ---- wave64 arg-reductions on (double value, uint32 index) without LDS traffic, with the serial
// tie rule (smallest value -- largest for MAX -- then the lowest index): the result is identical in
// every lane and independent of the schedule.  Values are compared through an order-preserving
// 64-bit key (sign-folded bits, -0 folded onto +0).  Its HIGH word is reduced with one DPP move and
// one v_min/max_u32 per step (quad_perm xor1, xor2, row_half_mirror (8), row_mirror (16), then the
// gfx950 v_permlane16_swap / v_permlane32_swap for the 32/64-lane halves); a ballot then finds the
// lanes holding the winning high word -- almost always exactly one, whose value, index and lane are
// read directly.  Only a tie of the high words costs a second 32-bit pass over the low words, and
// only an exact value tie a third pass for the lowest index.  (Replaces a 64-bit value pass plus an
// index pass on every reduction: about half the DPP steps.)
struct VI {
  double v;
  uint32_t i;
};
struct VIL {  // winner: value, index and the lane that holds it (read its other fields with readlane)
  double v;
  uint32_t i;
  int lane;
};

template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
  return uint32_t(__builtin_amdgcn_mov_dpp(int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ uint64_t order_key(double v) {
  const uint64_t u = uint64_t(__double_as_longlong(v == 0.0 ? 0.0 : v));
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
template <bool MIN>
__device__ __forceinline__ uint32_t pick32(uint32_t a, uint32_t b) {
  return MIN ? min(a, b) : max(a, b);
}
// v_permlane{16,32}_swap with both operands = x returns, in every lane, its own value and its
// partner's (in an order that depends on the row): combine both.
template <bool MIN, bool S32>
__device__ __forceinline__ uint32_t swap_pick32(uint32_t x) {
  if constexpr (S32) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return pick32<MIN>(r[0], r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return pick32<MIN>(r[0], r[1]);
  }
}
// Butterfly over aligned groups of L lanes (L = 1..64, power of two); returns lane 0's group result
// (wave-uniform).
template <bool MIN, int L>
__device__ __forceinline__ uint32_t group_pick32(uint32_t x) {
  if (L > 1) x = pick32<MIN>(x, dpp32<0xB1>(x));   // quad_perm [1,0,3,2]
  if (L > 2) x = pick32<MIN>(x, dpp32<0x4E>(x));   // quad_perm [2,3,0,1]
  if (L > 4) x = pick32<MIN>(x, dpp32<0x141>(x));  // row_half_mirror
  if (L > 8) x = pick32<MIN>(x, dpp32<0x140>(x));  // row_mirror
  if (L > 16) x = swap_pick32<MIN, false>(x);
  if (L > 32) x = swap_pick32<MIN, true>(x);
  return uint32_t(__builtin_amdgcn_readfirstlane(int(x)));
}
__device__ __forceinline__ double read_lane64(double x, int src) {
  return mk64(uint32_t(__builtin_amdgcn_readlane(int(lo32(x)), src)),
              uint32_t(__builtin_amdgcn_readlane(int(hi32(x)), src)));
}
// Inclusive prefix sum over the 64 lanes (lane L gets x[0] + ... + x[L]); full wave.  DPP only:
// Hillis-Steele inside each 16-lane row (row_shr 1, 2, 4, 8; lanes shifted in from outside the row
// read 0), then row_bcast:15 adds row 0's total to row 1 and row 2's to row 3, and row_bcast:31
// adds lane 31's (rows 0-1 total) to rows 2 and 3.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int32_t dpp_add_src(int32_t x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, ROW_MASK, 0xF, false);
}
__device__ __forceinline__ int32_t wave_incl_scan(int32_t x) {
  x += dpp_add_src<0x111>(x);  // row_shr:1
  x += dpp_add_src<0x112>(x);  // row_shr:2
  x += dpp_add_src<0x114>(x);  // row_shr:4
  x += dpp_add_src<0x118>(x);  // row_shr:8
  x += dpp_add_src<0x142, 0xA>(x);  // row_bcast:15 -> rows 1, 3
  x += dpp_add_src<0x143, 0xC>(x);  // row_bcast:31 -> rows 2, 3
  return x;
}
// a strictly before b in wave_arg's order: the value key (smallest for MIN, largest for MAX), then
// the lowest index.  A lane merging several candidates with it holds the one wave_arg would pick.
template <bool MIN>
__device__ __forceinline__ bool beats(VI a, VI b) {
  const uint64_t ka = order_key(a.v), kb = order_key(b.v);
  if (ka != kb) return MIN ? ka < kb : ka > kb;
  return a.i < b.i;
}
// Requires a full wave (EXEC = all 64 lanes).  L = number of leading lanes that may hold candidates;
// lanes >= L must hold "no candidate" sentinels (value +inf for MIN / -inf for MAX, index
// kSentinel), which never beat a real candidate.
template <bool MIN, int L = 64>
__device__ __forceinline__ VIL wave_arg(VI a) {
  const uint64_t k = order_key(a.v);
  const uint32_t kh = uint32_t(k >> 32), kl = uint32_t(k);
  const uint32_t bh = group_pick32<MIN, L>(kh);
  unsigned long long tie = __ballot(kh == bh);
  if (__popcll(tie) != 1) {  // equal high words: compare the low words
    const uint32_t bl = group_pick32<MIN, L>(kh == bh ? kl : (MIN ? 0xFFFFFFFFu : 0u));
    const bool same = kh == bh && kl == bl;
    tie = __ballot(same);
    if (__popcll(tie) != 1) {  // exact value tie (e.g. the first iteration, f = -y): lowest index
      const uint32_t bi = group_pick32<true, L>(same ? a.i : 0xFFFFFFFFu);
      tie = __ballot(same && a.i == bi);
    }
  }
  const int src = __builtin_ctzll(tie);
  return VIL{read_lane64(a.v, src), uint32_t(__builtin_amdgcn_readlane(int(a.i), src)), src};
}

// wave_arg's winning lane only (wave-uniform): the caller reads or publishes the winner's fields.
template <bool MIN, int L = 64>
__device__ __forceinline__ int wave_arg_lane(VI a) {
  const uint64_t k = order_key(a.v);
  const uint32_t kh = uint32_t(k >> 32), kl = uint32_t(k);
  const uint32_t bh = group_pick32<MIN, L>(kh);
  unsigned long long tie = __ballot(kh == bh);
  if (__popcll(tie) != 1) {
    const uint32_t bl = group_pick32<MIN, L>(kh == bh ? kl : (MIN ? 0xFFFFFFFFu : 0u));
    const bool same = kh == bh && kl == bl;
    tie = __ballot(same);
    if (__popcll(tie) != 1) {
      const uint32_t bi = group_pick32<true, L>(same ? a.i : 0xFFFFFFFFu);
      tie = __ballot(same && a.i == bi);
    }
  }
  return __builtin_ctzll(tie);
}

// Both of an iteration's wave arg-reductions in lockstep (minimum over I_high, maximum over I_low):
// the two high-word butterflies are independent DPP chains and interleave; each side falls back to
// wave_arg (low words, then the lowest index) only when its high word ties.  Same results as two
// wave_arg calls.
__device__ __forceinline__ void wave_arg_pair(VI mn, VI mx, VIL& rmn, VIL& rmx) {
  const uint32_t k1 = uint32_t(order_key(mn.v) >> 32), k2 = uint32_t(order_key(mx.v) >> 32);
  uint32_t a = k1, b = k2;
  a = min(a, dpp32<0xB1>(a));
  b = max(b, dpp32<0xB1>(b));
  a = min(a, dpp32<0x4E>(a));
  b = max(b, dpp32<0x4E>(b));
  a = min(a, dpp32<0x141>(a));
  b = max(b, dpp32<0x141>(b));
  a = min(a, dpp32<0x140>(a));
  b = max(b, dpp32<0x140>(b));
  a = swap_pick32<true, false>(a);
  b = swap_pick32<false, false>(b);
  a = swap_pick32<true, true>(a);
  b = swap_pick32<false, true>(b);
  const uint32_t h1 = uint32_t(__builtin_amdgcn_readfirstlane(int(a)));
  const uint32_t h2 = uint32_t(__builtin_amdgcn_readfirstlane(int(b)));
  const unsigned long long t1 = __ballot(k1 == h1), t2 = __ballot(k2 == h2);
  if (__popcll(t1) == 1) {
    const int src = __builtin_ctzll(t1);
    rmn = VIL{read_lane64(mn.v, src), uint32_t(__builtin_amdgcn_readlane(int(mn.i), src)), src};
  } else {
    rmn = wave_arg<true>(mn);
  }
  if (__popcll(t2) == 1) {
    const int src = __builtin_ctzll(t2);
    rmx = VIL{read_lane64(mx.v, src), uint32_t(__builtin_amdgcn_readlane(int(mx.i), src)), src};
  } else {
    rmx = wave_arg<false>(mx);
  }
}

// The lanes holding wave_arg<true>(mn) and wave_arg<false>(mx) (wave-uniform), with the two high-word
// butterflies interleaved; the caller's winning lanes publish their own fields.
__device__ __forceinline__ void wave_arg_pair_lanes(VI mn, VI mx, int& lmn, int& lmx) {
  const uint32_t k1 = uint32_t(order_key(mn.v) >> 32), k2 = uint32_t(order_key(mx.v) >> 32);
  uint32_t a = k1, b = k2;
  a = min(a, dpp32<0xB1>(a));
  b = max(b, dpp32<0xB1>(b));
  a = min(a, dpp32<0x4E>(a));
  b = max(b, dpp32<0x4E>(b));
  a = min(a, dpp32<0x141>(a));
  b = max(b, dpp32<0x141>(b));
  a = min(a, dpp32<0x140>(a));
  b = max(b, dpp32<0x140>(b));
  a = swap_pick32<true, false>(a);
  b = swap_pick32<false, false>(b);
  a = swap_pick32<true, true>(a);
  b = swap_pick32<false, true>(b);
  const uint32_t h1 = uint32_t(__builtin_amdgcn_readfirstlane(int(a)));
  const uint32_t h2 = uint32_t(__builtin_amdgcn_readfirstlane(int(b)));
  const unsigned long long t1 = __ballot(k1 == h1), t2 = __ballot(k2 == h2);
  lmn = __popcll(t1) == 1 ? __builtin_ctzll(t1) : wave_arg_lane<true>(mn);
  lmx = __popcll(t2) == 1 ? __builtin_ctzll(t2) : wave_arg_lane<false>(mx);
}

struct PersistShared {
  double wv[2][16], wa[2][16];  // per-wave candidates [min|max][wave]
  uint32_t wi[2][16];
  double gv[2], ga[2];          // global winners of the current epoch
  uint32_t gi[2];
  int timeout;
  int64_t rslot[2];             // cached row source: slots of rows (i_high, i_low) ...
  int32_t rmiss[2];             // ... and whether this epoch fills them
  double k12;                   // second-order selection: K(i_high, j) from the winner's record
};

// ---- Row sources of the persistent solver.  choose() runs on one lane of every workgroup once the
// pair is known (before the barrier that publishes it); fetch() then gives every thread the rows'
// values for its elements plus K11 / K22 / K12, issuing all loads in one memory round trip.
// Second-order selection reads the pair's rows one at a time (row i_high before the second exchange,
// row j after it): choose_one() (lane 0 of wave 0, `keep` = a slot that must survive) and fetch_one()
// (every thread: its elements of the row, and K(row, row)).
struct ResidentRows {  // the resident n x n Gram
  const double* __restrict__ K;
  int64_t ldk;
  __device__ __forceinline__ void choose(PersistShared&, uint32_t, uint32_t) const {}
  __device__ __forceinline__ void choose_one(PersistShared&, int, uint32_t, int64_t) const {}
  template <int NT, int E>
  __device__ __forceinline__ void fetch_one(const PersistShared&, int, int64_t row, int64_t lo, int t,
                                            int64_t hi_end, double (&k)[E], double& diag) const {
    const double* R = K + row * ldk;
    diag = R[row];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = lo + t + NT * e;
      k[e] = i < hi_end ? R[i] : 0.0;
    }
  }
  template <int NT, int E>
  __device__ __forceinline__ void fetch(const PersistShared&, int64_t ih, int64_t il, int64_t lo, int t,
                                        int64_t hi_end, double (&kh)[E], double (&kl)[E], double& K11,
                                        double& K22, double& K12) const {
    K11 = K[ih * ldk + ih];
    K22 = K[il * ldk + il];
    K12 = K[ih * ldk + il];
    const double* Kh = K + ih * ldk;
    const double* Kl = K + il * ldk;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = lo + t + NT * e;
      const bool ok = i < hi_end;
      kh[e] = ok ? Kh[i] : 0.0;
      kl[e] = ok ? Kl[i] : 0.0;
    }
  }
};

// K(ih, il) of the exact-integer path, computed redundantly by every wave: lane s takes k-step s
// (and s + 64), then the steps are combined in order with the igram group flushes -> kval bits.
// mid() runs after K12's own loads are issued and before their data is used: loads it issues
// (the hit path's row reads) stay in flight through K12's arithmetic, since the in-order vmcnt
// wait for K12's operands does not cover loads issued after them.  Needs q.kq <= 32 * 128.
template <class Mid>
__device__ __forceinline__ double k12_exact(const QRows& q, int64_t ih, int64_t il, double neg_gamma, Mid mid) {
  const int lane = threadIdx.x & 63, nsteps = q.kq / 32;
  int32_t d[2] = {0, 0};
  double wl[2] = {0.0, 0.0};  // step s's flush weight in lane s & 63 (no loads in the serial loop)
  int4 a0[2], a1[2], b0[2], b1[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int s = lane + 64 * r;
    if (s < q.main_step0) wl[r] = q.step_w[s];
    a0[r] = a1[r] = b0[r] = b1[r] = int4{0, 0, 0, 0};
    if (s < nsteps) {
      const int4* pa = reinterpret_cast<const int4*>(q.Q + ih * int64_t(q.kq)) + 2 * s;
      const int4* pb = reinterpret_cast<const int4*>(q.Q + il * int64_t(q.kq)) + 2 * s;
      a0[r] = pa[0];
      a1[r] = pa[1];
      b0[r] = pb[0];
      b1[r] = pb[1];
    }
  }
  const int32_t n0h = q.N0[ih], n0l = q.N0[il];
  const double wnh = q.main_step0 > 0 ? q.WN[ih] : 0.0, wnl = q.main_step0 > 0 ? q.WN[il] : 0.0;
  mid();
#pragma unroll
  for (int r = 0; r < 2; ++r) {  // zero operands past nsteps give d = 0
    int32_t acc = 0;
    acc = __builtin_amdgcn_sdot4(a0[r].x, b0[r].x, acc, false);
    acc = __builtin_amdgcn_sdot4(a0[r].y, b0[r].y, acc, false);
    acc = __builtin_amdgcn_sdot4(a0[r].z, b0[r].z, acc, false);
    acc = __builtin_amdgcn_sdot4(a0[r].w, b0[r].w, acc, false);
    acc = __builtin_amdgcn_sdot4(a1[r].x, b1[r].x, acc, false);
    acc = __builtin_amdgcn_sdot4(a1[r].y, b1[r].y, acc, false);
    acc = __builtin_amdgcn_sdot4(a1[r].z, b1[r].z, acc, false);
    acc = __builtin_amdgcn_sdot4(a1[r].w, b1[r].w, acc, false);
    d[r] = acc;
  }
  // kval's serial walk is "acc += d[s]; at a flush step: x += w * acc, acc = 0".  The integer
  // group sums are exact, so they come from an inclusive prefix scan over the steps (group sum
  // = P[flush] - P[previous flush]); only the FP64 accumulation stays serial, over the flush
  // steps alone and in step order -- the same operands in the same order as kval.
  const int32_t P0 = wave_incl_scan(d[0]);
  const int32_t P1 = nsteps > 64 ? wave_incl_scan(d[1]) + __builtin_amdgcn_readlane(P0, 63) : 0;
  uint64_t m0 = __ballot(lane < q.main_step0 && wl[0] != 0.0);
  uint64_t m1 = __ballot(lane + 64 < q.main_step0 && wl[1] != 0.0);
  int32_t prev = 0;
  double x = 0.0;
  while (m0) {
    const int s = __builtin_ctzll(m0);
    m0 &= m0 - 1;
    const int32_t ps = __builtin_amdgcn_readlane(P0, s);
    x = __builtin_fma(read_lane64(wl[0], s), double(ps - prev), x);
    prev = ps;
  }
  while (m1) {
    const int s = __builtin_ctzll(m1);
    m1 &= m1 - 1;
    const int32_t ps = __builtin_amdgcn_readlane(P1, s);
    x = __builtin_fma(read_lane64(wl[1], s), double(ps - prev), x);
    prev = ps;
  }
  const int32_t acc = __builtin_amdgcn_readlane(nsteps > 64 ? P1 : P0, 63) - prev;
  const int32_t D0 = n0h + n0l - 2 * acc;
  double dist = q.w0 * double(D0);
  if (q.main_step0 > 0) dist += (wnh + wnl) - 2.0 * x;
  dist = dist > 0.0 ? dist : 0.0;
  return exp(neg_gamma * dist);
}

// Kernel rows held in an HBM row cache of nslots x ldc doubles, computed from the rows themselves
// on a miss (qrows.h).  The 2-way set-associative directory (int32 tags + MRU way per set) lives
// in LDS and is REPLICATED in every workgroup: all workgroups see the same pair sequence and run the
// same deterministic lookups, so they agree on every slot and miss without exchanging anything.  On
// a miss each workgroup computes its own slice of the row (kval2: both rows of the pair in one pass
// over each element's quantised row) and writes it into the slot; hits read the slot, exactly like
// the resident Gram.  Values are bit-identical to the exact-integer Gram, hence the trajectory.
template <bool INT>
struct CachedRows {
  QRows q;
  double* __restrict__ cache;
  int64_t ldc;
  int32_t* tags;    // LDS, nslots entries (-1 = empty)
  uint8_t* mru;     // LDS, nslots / 2 entries
  int64_t nsets;
  double neg_gamma;

  __device__ __forceinline__ int64_t lookup(int64_t row, int64_t keep, int32_t* miss) const {
    const int64_t set = uint32_t(row) % uint32_t(nsets), s0 = 2 * set;  // row < 2^31, nsets <= 8192
    const int2 tw = reinterpret_cast<const int2*>(tags)[set];           // both ways in one LDS read
    if (tw.x == int32_t(row)) {
      mru[set] = 0;
      *miss = 0;
      return s0;
    }
    if (tw.y == int32_t(row)) {
      mru[set] = 1;
      *miss = 0;
      return s0 + 1;
    }
    int way = 1 - int(mru[set]);
    if (s0 + way == keep) way = 1 - way;
    tags[s0 + way] = int32_t(row);
    mru[set] = uint8_t(way);
    *miss = 1;
    return s0 + way;
  }
  __device__ __forceinline__ void choose_one(PersistShared& sh, int which, uint32_t row, int64_t keep) const {
    int32_t m = 0;
    sh.rslot[which] = lookup(row, keep, &m);
    sh.rmiss[which] = m;
  }
  template <int NT, int E>
  __device__ __forceinline__ void fetch_one(const PersistShared& sh, int which, int64_t row, int64_t lo, int t,
                                            int64_t hi_end, double (&k)[E], double& diag) const {
    diag = 1.0;  // kval(a, a)
    double* Cr = cache + sh.rslot[which] * ldc;
    if (sh.rmiss[which]) {
      if constexpr (INT) {
        constexpr int EG = E < 4 ? E : 4;
#pragma unroll 1
        for (int e0 = 0; e0 < E; e0 += EG) fill<NT, EG, true, false>(lo + int64_t(NT) * e0, row, row, t, hi_end, Cr, Cr);
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int64_t i = lo + t + NT * e;
          if (i < hi_end) Cr[i] = kval<false>(q, row, i, neg_gamma);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {  // this thread's own stores, or a filled slot from an earlier epoch
      const int64_t i = lo + t + NT * e;
      k[e] = i < hi_end ? Cr[i] : 0.0;
    }
  }
  __device__ __forceinline__ void choose(PersistShared& sh, uint32_t ih, uint32_t il) const {
    int32_t mh = 0, ml = 0;
    const int64_t sh_ = lookup(ih, -1, &mh);
    const int64_t sl_ = lookup(il, sh_, &ml);
    sh.rslot[0] = sh_;
    sh.rslot[1] = sl_;
    sh.rmiss[0] = mh;
    sh.rmiss[1] = ml;
  }
  template <class Mid>
  __device__ __forceinline__ double k12(int64_t ih, int64_t il, Mid mid) const {
    if constexpr (INT) {
      return k12_exact(q, ih, il, neg_gamma, mid);
    } else {
      mid();
      return kval<false>(q, ih, il, neg_gamma);
    }
  }
  template <int NT, int E>
  __device__ __forceinline__ void fetch(const PersistShared& sh, int64_t ih, int64_t il, int64_t lo, int t,
                                        int64_t hi_end, double (&kh)[E], double (&kl)[E], double& K11,
                                        double& K22, double& K12) const {
    const int32_t mh = sh.rmiss[0], ml = sh.rmiss[1];
    double* Ch = cache + sh.rslot[0] * ldc;
    double* Cl = cache + sh.rslot[1] * ldc;
    K11 = 1.0;  // kval(a, a): the Gram's diagonal is exactly 1
    K22 = 1.0;
    if constexpr (INT) {
      if (!(mh | ml)) {  // hit: the row reads overlap K12's arithmetic
        K12 = k12(ih, il, [&] {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const int64_t i = lo + t + NT * e;
            const bool ok = i < hi_end;
            kh[e] = ok ? Ch[i] : 0.0;
            kl[e] = ok ? Cl[i] : 0.0;
          }
        });
        return;
      }
      K12 = k12(ih, il, [] {});
      // A miss first writes this thread's elements of the missed row(s) into the slot, in groups of
      // EG elements with the group loop kept rolled, so the fill's registers do not stack on the
      // E-element solver state; then every element is read back from the slot like a hit (a
      // thread reading its own stores).
      constexpr int EG = E < 4 ? E : 4;
#pragma unroll 1
      for (int e0 = 0; e0 < E; e0 += EG) {
        if (mh && ml)
          fill<NT, EG, true, true>(lo + int64_t(NT) * e0, ih, il, t, hi_end, Ch, Cl);
        else if (mh)
          fill<NT, EG, true, false>(lo + int64_t(NT) * e0, ih, il, t, hi_end, Ch, Cl);
        else
          fill<NT, EG, false, true>(lo + int64_t(NT) * e0, ih, il, t, hi_end, Ch, Cl);
      }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int64_t i = lo + t + NT * e;
        const bool ok = i < hi_end;
        kh[e] = ok ? Ch[i] : 0.0;
        kl[e] = ok ? Cl[i] : 0.0;
      }
      return;
    }
    K12 = k12(ih, il, [] {});
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = lo + t + NT * e;
      const bool ok = i < hi_end;
      kh[e] = (ok && !mh) ? Ch[i] : 0.0;
      kl[e] = (ok && !ml) ? Cl[i] : 0.0;
    }
    if (mh | ml) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int64_t i = lo + t + NT * e;
        if (i < hi_end) {
          double a, b;
          kval2<INT>(q, ih, il, i, neg_gamma, &a, &b);
          if (mh) {
            kh[e] = a;
            Ch[i] = a;
          }
          if (ml) {
            kl[e] = b;
            Cl[i] = b;
          }
        }
      }
    }
  }
  // Miss fill of the exact-integer rows for this thread's E elements: the k-step loop is outermost,
  // so every step issues the loads of all E elements' chunks at once (E-fold memory parallelism
  // against the one-element-at-a-time walk of kval2) -- per element the arithmetic and its order
  // are kval's, so the values are bit-identical.  DA / DB: rows ih / il missed.  Elements
  // lo + t + NT * e, e < EG.
  template <int NT, int EG, bool DA, bool DB>
  __device__ __forceinline__ void fill(int64_t lo, int64_t ih, int64_t il, int t, int64_t hi_end, double* Ch,
                                       double* Cl) const {
    const int4* pa = reinterpret_cast<const int4*>(q.Q + ih * int64_t(q.kq));
    const int4* pb = reinterpret_cast<const int4*>(q.Q + il * int64_t(q.kq));
    const int4* pq = q.Qt ? reinterpret_cast<const int4*>(q.Qt) : nullptr;
    const int64_t cs = q.Qt ? q.n_rows : 1;  // chunk stride (interleaved) or 1 (row-major rows)
    int32_t acca[EG], accb[EG];
    double xa[EG], xb[EG];
    const int4* pi[EG];
#pragma unroll
    for (int e = 0; e < EG; ++e) {
      const int64_t i = lo + t + NT * e;
      const int64_t ic = i < hi_end ? i : lo;  // clamped (valid) row for the tail's dummy loads
      pi[e] = pq ? pq + ic : reinterpret_cast<const int4*>(q.Q + ic * int64_t(q.kq));
      acca[e] = accb[e] = 0;
      xa[e] = xb[e] = 0.0;
    }
    const int nsteps = q.kq / 32;
    int4 c0[EG], c1[EG];
    for (int s = 0; s < nsteps; ++s) {
#pragma unroll
      for (int e = 0; e < EG; ++e) {
        c0[e] = pi[e][(2 * s) * cs];
        c1[e] = pi[e][(2 * s + 1) * cs];
      }
      int4 a0, a1, b0, b1;
      if (DA) {
        a0 = pa[2 * s];
        a1 = pa[2 * s + 1];
      }
      if (DB) {
        b0 = pb[2 * s];
        b1 = pb[2 * s + 1];
      }
#pragma unroll
      for (int e = 0; e < EG; ++e) {
        if (DA) {
          int32_t acc = acca[e];
          acc = __builtin_amdgcn_sdot4(a0.x, c0[e].x, acc, false);
          acc = __builtin_amdgcn_sdot4(a0.y, c0[e].y, acc, false);
          acc = __builtin_amdgcn_sdot4(a0.z, c0[e].z, acc, false);
          acc = __builtin_amdgcn_sdot4(a0.w, c0[e].w, acc, false);
          acc = __builtin_amdgcn_sdot4(a1.x, c1[e].x, acc, false);
          acc = __builtin_amdgcn_sdot4(a1.y, c1[e].y, acc, false);
          acc = __builtin_amdgcn_sdot4(a1.z, c1[e].z, acc, false);
          acca[e] = __builtin_amdgcn_sdot4(a1.w, c1[e].w, acc, false);
        }
        if (DB) {
          int32_t acc = accb[e];
          acc = __builtin_amdgcn_sdot4(b0.x, c0[e].x, acc, false);
          acc = __builtin_amdgcn_sdot4(b0.y, c0[e].y, acc, false);
          acc = __builtin_amdgcn_sdot4(b0.z, c0[e].z, acc, false);
          acc = __builtin_amdgcn_sdot4(b0.w, c0[e].w, acc, false);
          acc = __builtin_amdgcn_sdot4(b1.x, c1[e].x, acc, false);
          acc = __builtin_amdgcn_sdot4(b1.y, c1[e].y, acc, false);
          acc = __builtin_amdgcn_sdot4(b1.z, c1[e].z, acc, false);
          accb[e] = __builtin_amdgcn_sdot4(b1.w, c1[e].w, acc, false);
        }
      }
      if (s < q.main_step0) {
        const double wg = q.step_w[s];
        if (wg != 0.0) {  // igram_tri_kernel's group flush, same order and expression
#pragma unroll
          for (int e = 0; e < EG; ++e) {
            if (DA) {
              xa[e] = __builtin_fma(wg, double(acca[e]), xa[e]);
              acca[e] = 0;
            }
            if (DB) {
              xb[e] = __builtin_fma(wg, double(accb[e]), xb[e]);
              accb[e] = 0;
            }
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < EG; ++e) {
      const int64_t i = lo + t + NT * e;
      if (i >= hi_end) continue;
      if (DA) {
        double dist = q.w0 * double(q.N0[ih] + q.N0[i] - 2 * acca[e]);
        if (q.main_step0 > 0) dist += (q.WN[ih] + q.WN[i]) - 2.0 * xa[e];
        dist = dist > 0.0 ? dist : 0.0;
        Ch[i] = ih == i ? 1.0 : exp(neg_gamma * dist);
      }
      if (DB) {
        double dist = q.w0 * double(q.N0[il] + q.N0[i] - 2 * accb[e]);
        if (q.main_step0 > 0) dist += (q.WN[il] + q.WN[i]) - 2.0 * xb[e];
        dist = dist > 0.0 ? dist : 0.0;
        Cl[i] = il == i ? 1.0 : exp(neg_gamma * dist);
      }
    }
  }
};

// Distributed SMO row source (dsmo.hip): this team's slab K(:, [col0, col0 + ldw)) holds the rows'
// entries of the team's own points; K11 = K22 = 1 (the Gram's diagonal) and K12 = K(ih, il), which
// may lie in another team's slab, is computed from the two quantised rows with the Gram's exact
// arithmetic (k12_exact) while the slab loads are in flight -- the same kernel values as the
// resident Gram, hence the same trajectory.  First-order selection only.
struct SlabRows {
  const double* __restrict__ K;
  int64_t ldw, col0;
  QRows q;
  double neg_gamma;
  __device__ __forceinline__ void choose(PersistShared&, uint32_t, uint32_t) const {}
  template <int NT, int E>
  __device__ __forceinline__ void fetch(const PersistShared&, int64_t ih, int64_t il, int64_t lo, int t,
                                        int64_t hi_end, double (&kh)[E], double (&kl)[E], double& K11,
                                        double& K22, double& K12) const {
    K11 = 1.0;
    K22 = 1.0;
    const double* Kh = K + ih * ldw - col0;
    const double* Kl = K + il * ldw - col0;
    K12 = k12_exact(q, ih, il, neg_gamma, [&] {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int64_t i = lo + t + NT * e;
        const bool ok = i < hi_end;
        kh[e] = ok ? Kh[i] : 0.0;
        kl[e] = ok ? Kl[i] : 0.0;
      }
    });
  }
};

// Diagnostic build (STAMP = true, SVM355_PSMO_STAMP=1): workgroup 0 / lane 0 accumulates
// s_memtime deltas per phase over epochs [kStampFrom, kStampFrom + kStampCount) into stamps[0..7]
// (stamps[7] = s_memrealtime delta, 100 MHz, for the clock).  Never used in timed runs.
constexpr uint32_t kStampFrom = 200, kStampCount = 2000;
// Exchange-skew diagnostic (same STAMP builds): s_memrealtime (100 MHz, one clock for the whole chip)
// of every workgroup's record publication and of workgroup 0's sweep completion, for kSkewEpochs
// epochs from kStampFrom, at stamps[kSkewBase + g * kSkewEpochs + e] / [... + kMaxG * kSkewEpochs + e].
constexpr uint32_t kSkewEpochs = 64;
constexpr int kSkewBase = 16;
#define PSTAMP(k)                                                                   \
  do {                                                                              \
    if (STAMP && stamping) {                                                        \
      __builtin_amdgcn_sched_barrier(0);                                            \
      unsigned long long ts_;                                                       \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts_)::"memory");   \
      __builtin_amdgcn_sched_barrier(0);                                            \
      sacc[k] += ts_ - sprev;                                                       \
      sprev = ts_;                                                                  \
    }                                                                               \
  } while (0)

// XCD-local registration window (s_memrealtime ticks, 100 MHz): 2 ms, then the host falls back.
constexpr unsigned long long kRegisterTicks = 200000;

// One solve of the persistent SMO by G co-resident workgroups (this one is g), NT threads per
// workgroup (NW = NT/64 waves), E register-resident elements per thread: element e of thread t is
// training point lo + t + NT*e of the workgroup's slice.  Epochs continue from epoch0 (record tags
// must never repeat on a slot array); returns the last epoch used.  RPL = records per sweep lane:
// G <= 64 * RPL workgroups (lane L of wave 0 polls records L, L + 64, ...; slot arrays of 64 * RPL
// records per epoch parity).  The exchange-skew stamps exist for RPL = 1 only.
// WSS2 (opt-in, resident Gram, RPL = 1): second-order choice of the second index (smo_cpu.cpp):
// after the first exchange names i_high (and the first-order maximum for the stop test), every
// workgroup reads its slice of row i_high, computes -(f_t - f_ih)^2 / a_t over its I_low points
// above f_ih, and a second exchange (the next epoch) picks the minimum; its record carries the
// gain, j, alpha_j, f_j and K(i_high, j) (from the owner's row slice).
//
// PEER (distributed SMO, dsmo.hip): the G workgroups form teams that may run on different GPUs.
// Records go to the receive array of EVERY team (px.arr[0 .. px.n), system-scope stores into
// uncached fine-grained memory, local or a peer's over xGMI) as self-validating granules
// (peer_word); each workgroup sweeps its own team's array (px.own) with system-scope loads.
// g_state: the workgroup that writes the final state block (each team's first).
template <int NT, int E, bool STAMP, bool XLOCAL, class Rows, int RPL = 1, bool WSS2 = false, bool PEER = false>
__device__ __forceinline__ uint32_t persist_solve(
    PersistShared& sh, int G, int g, uint32_t epoch0, const Rows& rows,
    const int32_t* __restrict__ y, double* __restrict__ alpha, double* __restrict__ f, int64_t n, int64_t slice,
    unsigned long long* __restrict__ slots, SmoState* __restrict__ st, double C, double eps, double tau,
    int64_t max_iter, int64_t* __restrict__ trace, int64_t trace_cap, unsigned* __restrict__ err,
    int64_t spin_limit, unsigned long long* __restrict__ stamps, const PeerExch& px = PeerExch{}, int g_state = 0) {
  static_assert(!(PEER && (WSS2 || XLOCAL || STAMP)), "the peer exchange is first-order, device-wide, unstamped");
  constexpr int NW = NT / 64;
  unsigned long long sacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sprev = 0, rt0 = 0;
  bool stamping = false;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t lo = int64_t(g) * slice, hi_end = std::min<int64_t>(n, lo + slice);
  const double c_hi = C - eps, c_lo = 0.0 + eps;
  const double inf = __builtin_inf();

  double fr[E], ar[E];
  int32_t yr[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int64_t i = lo + t + NT * e;
    const bool ok = i < hi_end;
    fr[e] = ok ? f[i] : 0.0;
    ar[e] = ok ? alpha[i] : 0.0;
    yr[e] = ok ? y[i] : 0;  // y = 0 is in neither set
  }
  if (t == 0) sh.timeout = 0;
  int64_t num_iter = st->num_iter;
  double b_high = st->b_high, b_low = st->b_low;
  int32_t stop = SVM_STOP_RUNNING;

  uint32_t epoch = epoch0 + 1;
  for (;; ++epoch) {
    if (STAMP) {
      // window start: stamps[8] when the host set it (SVM355_PSMO_STAMP_FROM), else kStampFrom
      const uint32_t from = stamps[8] ? uint32_t(stamps[8]) : kStampFrom;
      const bool on = g == 0 && threadIdx.x == 0 && epoch >= from && epoch < from + kStampCount;
      if (on && !stamping) rt0 = __builtin_amdgcn_s_memrealtime();
      if (!on && stamping) sacc[7] = __builtin_amdgcn_s_memrealtime() - rt0;
      stamping = on;
      if (stamping) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(sprev)::"memory");
    }
    // ---- 1. local selection over the register slice (ascending index within a thread)
    // branch-free: selects, not exec-mask branches, over the E points
    VI mn{inf, kSentinel}, mx{-inf, kSentinel};
    double amn = 0.0, amx = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t i = uint32_t(lo + t + NT * e);
      const double a = ar[e], fi = fr[e];
      const int32_t yi = yr[e];
      const bool in_high = ((yi == 1) & (a < c_hi)) | ((yi == -1) & (a > c_lo));
      const bool in_low = ((yi == 1) & (a > c_lo)) | ((yi == -1) & (a < c_hi));
      const bool ch = in_high & (fi < mn.v), cl = in_low & (fi > mx.v);
      mn.v = ch ? fi : mn.v;
      mn.i = ch ? i : mn.i;
      amn = ch ? a : amn;
      mx.v = cl ? fi : mx.v;
      mx.i = cl ? i : mx.i;
      amx = cl ? a : amx;
    }
    {
      // both reductions interleaved; the winning lanes publish their own value, index and alpha
      int lmn, lmx;
      wave_arg_pair_lanes(mn, mx, lmn, lmx);
      PSTAMP(0);
      if (lane == lmn) {
        sh.wv[0][w] = mn.v;
        sh.wi[0][w] = mn.i;
        sh.wa[0][w] = amn;
      }
      if (lane == lmx) {
        sh.wv[1][w] = mx.v;
        sh.wi[1][w] = mx.i;
        sh.wa[1][w] = amx;
      }
    }
    __syncthreads();
    PSTAMP(1);
    const size_t par_off = (size_t(epoch & 1) * (64 * RPL)) * kRecStride;
    unsigned long long* rec = (PEER ? px.arr[px.own] : slots) + par_off;
    if (w == 0) {
      // ---- 2. merge the NW waves and publish this workgroup's record (lanes 0..9, one granule each)
      VI a{inf, kSentinel}, b{-inf, kSentinel};
      double aa = 0.0, ba = 0.0;
      if (NW == 1) {
        a = VI{sh.wv[0][0], sh.wi[0][0]};
        b = VI{sh.wv[1][0], sh.wi[1][0]};
        aa = sh.wa[0][0];
        ba = sh.wa[1][0];
      } else {
        VI ca{inf, kSentinel}, cb{-inf, kSentinel};
        double caa = 0.0, cba = 0.0;
        if (lane < NW) {
          ca = VI{sh.wv[0][lane], sh.wi[0][lane]};
          cb = VI{sh.wv[1][lane], sh.wi[1][lane]};
          caa = sh.wa[0][lane];
          cba = sh.wa[1][lane];
        }
        // Lanes 0..NW-1 hold the wave results (sentinels above): log2(NW) steps; the winner is read
        // from its lane, so every publishing lane sees the same record.
        const VIL ra = wave_arg<true, NW>(ca), rb = wave_arg<false, NW>(cb);
        a = VI{ra.v, ra.i};
        b = VI{rb.v, rb.i};
        aa = read_lane64(caa, ra.lane);
        ba = read_lane64(cba, rb.lane);
      }
      if (lane < kGranules) {
        // Branch-free payload selection (no divergent switch).
        uint32_t pay = lo32(a.v);
        pay = lane == 1 ? hi32(a.v) : pay;
        pay = lane == 2 ? a.i : pay;
        pay = lane == 3 ? lo32(aa) : pay;
        pay = lane == 4 ? hi32(aa) : pay;
        pay = lane == 5 ? lo32(b.v) : pay;
        pay = lane == 6 ? hi32(b.v) : pay;
        pay = lane == 7 ? b.i : pay;
        pay = lane == 8 ? lo32(ba) : pay;
        pay = lane == 9 ? hi32(ba) : pay;
        // Memory-model note (XLOCAL).  The readers are other workgroups, but every participant runs
        // on XCD 0 (xcd_register checks HW_REG_XCC_ID), and HIP has no scope between workgroup and
        // agent.  On gfx950 the scopes differ only in the store's cache-coherence bits: workgroup
        // scope emits `global_store_dwordx2 ... sc0` (through the write-through vL1D into the
        // XCD's L2), agent scope `... sc1` (written through past the XCD-local L2 to the
        // device-coherent level, because the eight XCD L2s are not coherent with each other).  The
        // pollers' agent-scope loads (`global_load_dwordx2 ... sc1`) miss the vL1D and are served by
        // that same L2, the single point of coherence of one XCD, so the sc0 store is visible to
        // them.  Agent scope costs 16 % at the headline shape (3.42 -> 3.95 us/iter at n = 60k,
        // profiles/r2_psmo_store_scope_ab.txt); tests/test_isa_pins.py pins both encodings.
        if constexpr (PEER) {
          const unsigned long long word = peer_word(epoch, pay);
          const size_t off = par_off + size_t(g) * kRecStride + lane;
#pragma unroll
          for (int k = 0; k < kMaxPeers; ++k)
            if (k < px.n) __hip_atomic_store(px.arr[k] + off, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else if constexpr (XLOCAL) {
          __hip_atomic_store(rec + size_t(g) * kRecStride + lane, (uint64_t(epoch) << 32) | pay, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          __hip_atomic_store(rec + size_t(g) * kRecStride + lane, (uint64_t(epoch) << 32) | pay, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      PSTAMP(2);
      if (STAMP && RPL == 1 && lane == 0 && epoch >= kStampFrom && epoch < kStampFrom + kSkewEpochs)
        stamps[kSkewBase + g * kSkewEpochs + (epoch - kStampFrom)] = __builtin_amdgcn_s_memrealtime();
      // ---- 3. lane L polls the records of workgroups L, L + 64, ... until their ten tags equal the
      // epoch (every spin round re-reads all of them: one round trip, not one per record), then
      // keeps the best of them under wave_arg's order (value key, then the lowest index)
      VI gm{inf, kSentinel}, gx{-inf, kSentinel};
      double agm = 0.0, agx = 0.0;
      bool timed_out = false;
      if (lane < G) {
        uint32_t v[RPL][kGranules];
        // PEER: spin_limit is a wall-clock bound in s_memrealtime ticks (100 MHz), not a poll count
        const unsigned long long t_spin0 = PEER ? __builtin_amdgcn_s_memrealtime() : 0ull;
        for (int64_t spins = 0;; ++spins) {
          bool ok = true;
#pragma unroll
          for (int rr = 0; rr < RPL; ++rr) {
            if (RPL == 1 || lane + 64 * rr < G) {
              const unsigned long long* r = rec + size_t(lane + 64 * rr) * kRecStride;
#pragma unroll
              for (int k = 0; k < kGranules; ++k) {
                if constexpr (PEER) {
                  const unsigned long long x = __hip_atomic_load(r + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                  v[rr][k] = uint32_t(x);
                  ok &= peer_valid(x, epoch);
                } else {
                  const unsigned long long x = __hip_atomic_load(r + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                  v[rr][k] = uint32_t(x);
                  ok &= uint32_t(x >> 32) == epoch;
                }
              }
            }
          }
          if (ok) break;
          if (PEER ? int64_t(__builtin_amdgcn_s_memrealtime() - t_spin0) > spin_limit : spins > spin_limit) {
            timed_out = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (!timed_out) {
#pragma unroll
          for (int rr = 0; rr < RPL; ++rr) {
            if (RPL == 1 || lane + 64 * rr < G) {
              const VI cm{mk64(v[rr][0], v[rr][1]), v[rr][2]}, cx{mk64(v[rr][5], v[rr][6]), v[rr][7]};
              if (rr == 0 || beats<true>(cm, gm)) {
                gm = cm;
                agm = mk64(v[rr][3], v[rr][4]);
              }
              if (rr == 0 || beats<false>(cx, gx)) {
                gx = cx;
                agx = mk64(v[rr][8], v[rr][9]);
              }
            }
          }
        }
      }
      const bool any_to = __any(timed_out);
      if (STAMP && RPL == 1 && g == 0 && lane == 0 && epoch >= kStampFrom && epoch < kStampFrom + kSkewEpochs)
        stamps[kSkewBase + kMaxG * kSkewEpochs + (epoch - kStampFrom)] = __builtin_amdgcn_s_memrealtime();
      PSTAMP(3);
      VIL wgm, wgx;
      wave_arg_pair(gm, gx, wgm, wgx);  // the two reductions interleaved
      const double awgm = read_lane64(agm, wgm.lane), awgx = read_lane64(agx, wgx.lane);
      if (lane == 0) {
        sh.gv[0] = wgm.v;
        sh.gi[0] = wgm.i;
        sh.ga[0] = awgm;
        sh.gv[1] = wgx.v;
        sh.gi[1] = wgx.i;
        sh.ga[1] = awgx;
        // a pair that will be updated: the row source prepares its rows (every workgroup alike;
        // second-order selection: row i_high now, the second row after the second exchange)
        if (!any_to && wgm.i != kSentinel && wgx.i != kSentinel && !(wgx.v <= wgm.v + 2.0 * tau)) {
          if constexpr (WSS2)
            rows.choose_one(sh, 0, wgm.i, -1);
          else
            rows.choose(sh, wgm.i, wgx.i);
        }
        if (any_to) {
          sh.timeout = 1;
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    __syncthreads();
    PSTAMP(4);
    if (sh.timeout) {
      stop = -1;
      break;
    }
    const uint32_t uih = sh.gi[0], uil = sh.gi[1];
    // ---- 4. stop tests and the two-variable update (identical in every workgroup)
    if (uih == kSentinel || uil == kSentinel) {
      stop = SVM_STOP_NO_CANDIDATE;
      break;
    }
    const int64_t ih = uih;
    int64_t il = uil;
    const double bh = sh.gv[0], bl = sh.gv[1];
    b_high = bh;
    b_low = bl;
    if (bl <= bh + 2.0 * tau) {
      stop = SVM_STOP_CONVERGED;
      break;
    }
    double K11, K22, K12;
    double kh[E], kl[E];
    int32_t yh, yl;
    double bl_upd = bl, al = sh.ga[1];  // the second index's f and alpha in the update
    if constexpr (WSS2) {
      // ---- 4b. row i_high, the local second-order candidate, a second exchange for j
      rows.template fetch_one<NT, E>(sh, 0, ih, lo, t, hi_end, kh, K11);
      VI cm{inf, kSentinel};
      double ca = 0.0, cf = 0.0, ck = 0.0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double a = ar[e], ft = fr[e];
        const int32_t yt = yr[e];
        const bool in_low = (yt == 1 && a > c_lo) || (yt == -1 && a < c_hi);
        if (!in_low || !(ft > bh)) continue;
        const double bb = ft - bh;
        double at = K11 + 1.0 - 2.0 * kh[e];  // K(t, t) = 1 for the RBF kernel
        if (at <= 0.0) at = eps;
        const double gain = -(bb * bb) / at;
        if (gain < cm.v) {  // ascending index within a thread: strict compare keeps the lowest
          cm = VI{gain, uint32_t(lo + t + NT * e)};
          ca = a;
          cf = ft;
          ck = kh[e];
        }
      }
      {
        const VIL wc = wave_arg<true>(cm);
        const double wa = read_lane64(ca, wc.lane), wf = read_lane64(cf, wc.lane), wk = read_lane64(ck, wc.lane);
        if (lane == 0) {
          sh.wv[0][w] = wc.v;
          sh.wi[0][w] = wc.i;
          sh.wa[0][w] = wa;
          sh.wv[1][w] = wf;
          sh.wa[1][w] = wk;
        }
      }
      __syncthreads();
      ++epoch;  // the second exchange's tags (records alternate parity buffers per exchange)
      unsigned long long* rec2 = slots + (size_t(epoch & 1) * (64 * RPL)) * kRecStride;
      if (w == 0) {
        VI a{inf, kSentinel};
        double aa = 0.0, af = 0.0, ak = 0.0;
        {
          VI c{inf, kSentinel};
          double c_a = 0.0, c_f = 0.0, c_k = 0.0;
          if (lane < NW) {
            c = VI{sh.wv[0][lane], sh.wi[0][lane]};
            c_a = sh.wa[0][lane];
            c_f = sh.wv[1][lane];
            c_k = sh.wa[1][lane];
          }
          const VIL r = wave_arg<true, NW>(c);
          a = VI{r.v, r.i};
          aa = read_lane64(c_a, r.lane);
          af = read_lane64(c_f, r.lane);
          ak = read_lane64(c_k, r.lane);
        }
        if (lane < kGranules) {
          uint32_t pay = lo32(a.v);
          pay = lane == 1 ? hi32(a.v) : pay;
          pay = lane == 2 ? a.i : pay;
          pay = lane == 3 ? lo32(aa) : pay;
          pay = lane == 4 ? hi32(aa) : pay;
          pay = lane == 5 ? lo32(af) : pay;
          pay = lane == 6 ? hi32(af) : pay;
          pay = lane == 7 ? a.i : pay;
          pay = lane == 8 ? lo32(ak) : pay;
          pay = lane == 9 ? hi32(ak) : pay;
          if constexpr (XLOCAL)  // same scope rule as the first exchange (memory-model note above)
            __hip_atomic_store(rec2 + size_t(g) * kRecStride + lane, (uint64_t(epoch) << 32) | pay, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
          else
            __hip_atomic_store(rec2 + size_t(g) * kRecStride + lane, (uint64_t(epoch) << 32) | pay, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        VI gm{inf, kSentinel};
        double ga = 0.0, gf = 0.0, gk = 0.0;
        bool timed_out = false;
        if (lane < G) {  // lane L: records L, L + 64, ... (as in the first exchange)
          uint32_t v[RPL][kGranules];
          for (int64_t spins = 0;; ++spins) {
            bool ok = true;
#pragma unroll
            for (int rr = 0; rr < RPL; ++rr) {
              if (RPL == 1 || lane + 64 * rr < G) {
                const unsigned long long* r = rec2 + size_t(lane + 64 * rr) * kRecStride;
#pragma unroll
                for (int k = 0; k < kGranules; ++k) {
                  const unsigned long long x = __hip_atomic_load(r + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                  v[rr][k] = uint32_t(x);
                  ok &= uint32_t(x >> 32) == epoch;
                }
              }
            }
            if (ok) break;
            if (spins > spin_limit) {
              timed_out = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          if (!timed_out) {
#pragma unroll
            for (int rr = 0; rr < RPL; ++rr) {
              if (RPL == 1 || lane + 64 * rr < G) {
                const VI c{mk64(v[rr][0], v[rr][1]), v[rr][2]};
                if (rr == 0 || beats<true>(c, gm)) {
                  gm = c;
                  ga = mk64(v[rr][3], v[rr][4]);
                  gf = mk64(v[rr][5], v[rr][6]);
                  gk = mk64(v[rr][8], v[rr][9]);
                }
              }
            }
          }
        }
        const bool any_to2 = __any(timed_out);
        const VIL wgm = wave_arg<true>(gm);
        const double wga = read_lane64(ga, wgm.lane), wgf = read_lane64(gf, wgm.lane), wgk = read_lane64(gk, wgm.lane);
        if (lane == 0) {
          sh.gi[1] = wgm.i;
          sh.ga[1] = wga;
          sh.gv[1] = wgf;
          sh.k12 = wgk;
          if (!any_to2 && wgm.i != kSentinel) rows.choose_one(sh, 1, wgm.i, sh.rslot[0]);  // keep row i_high
          if (any_to2) {
            sh.timeout = 1;
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      __syncthreads();
      if (sh.timeout) {
        stop = -1;
        break;
      }
      il = sh.gi[1];  // exists: the first-order i_low lies above f_ih + 2 tau
      bl_upd = sh.gv[1];
      al = sh.ga[1];
      K12 = sh.k12;
      rows.template fetch_one<NT, E>(sh, 1, il, lo, t, hi_end, kl, K22);
      yh = y[ih];
      yl = y[il];
    } else {
      // One memory round trip: scalars + this slice of rows i_high and i_low.
      yh = y[ih];
      yl = y[il];
      rows.template fetch<NT, E>(sh, ih, il, lo, t, hi_end, kh, kl, K11, K22, K12);
    }
    PSTAMP(5);
    const double ah = sh.ga[0];
    const int s = yh * yl;
    const double eta = K11 + K22 - 2.0 * K12;
    double U, V;
    if (s == -1) {
      U = fmax(0.0, al - ah);
      V = fmin(C, C + al - ah);
    } else {
      U = fmax(0.0, al + ah - C);
      V = fmin(C, al + ah);
    }
    if (!(U <= V + 1e-12)) {
      stop = SVM_STOP_INFEASIBLE;
      break;
    }
    if (eta <= eps) {
      stop = SVM_STOP_NONPOS_ETA;
      break;
    }
    double al_new = al + double(yl) * (bh - bl_upd) / eta;
    if (al_new > V) al_new = V;
    if (al_new < U) al_new = U;
    const double ah_new = ah + double(s) * (al - al_new);
    const double ch = (ah_new - ah) * double(yh);
    const double cl = (al_new - al) * double(yl);
    // ---- 5. apply: f for the whole slice, alpha for the owners
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = lo + t + NT * e;
      fr[e] += ch * kh[e] + cl * kl[e];  // main3.cpp:274 operation order
      if (i == ih) ar[e] = ah_new;
      if (i == il) ar[e] = al_new;
    }
    PSTAMP(6);
    if (g == 0 && t == 0 && trace && num_iter - 1 < trace_cap) {
      trace[2 * (num_iter - 1)] = ih;
      trace[2 * (num_iter - 1) + 1] = il;
    }
    ++num_iter;
    if (num_iter > max_iter) {
      stop = SVM_STOP_MAX_ITER;
      break;
    }
  }
  // Write the slice back; workgroup 0 publishes the final state (visible at kernel end).
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int64_t i = lo + t + NT * e;
    if (i < hi_end) {
      f[i] = fr[e];
      alpha[i] = ar[e];
    }
  }
  if (STAMP && g == 0 && t == 0)
    for (int k = 0; k < 8; ++k) stamps[k] = sacc[k];
  if (g == g_state && t == 0) {
    st->num_iter = num_iter;
    st->b_high = b_high;
    st->b_low = b_low;
    st->pending = 0;
    st->stop = stop < 0 ? SVM_STOP_RUNNING : stop;
  }
  return epoch;
}


// XCD-local team registration (thread 0 of a workgroup running on XCD `xcc`).  reg[0] counts the
// workgroups that landed on the team's XCD: the first glocal take ranks 0..glocal-1 and wait until
// all have registered, for at most kRegisterTicks.  The outcome is one compare-and-swap on the
// decision word reg[1] (0 forming, 1 go, 2 abandoned), so all participants agree even when the last
// one registers just as another gives up.  Returns the rank, -1 (not a participant) or -2
// (abandoned: *err = 2, nothing touched).
__device__ int xcd_register(unsigned* reg, unsigned* err, int glocal, unsigned long long ticks) {
  const unsigned tk = __hip_atomic_fetch_add(reg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tk >= unsigned(glocal)) return -1;
  unsigned* decision = reg + 1;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  unsigned d;
  while ((d = __hip_atomic_load(decision, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u) {
    unsigned want = 0u;
    if (__hip_atomic_load(reg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= unsigned(glocal))
      __hip_atomic_compare_exchange_strong(decision, &want, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    else if (__builtin_amdgcn_s_memrealtime() - t_start > ticks)
      __hip_atomic_compare_exchange_strong(decision, &want, 2u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    else
      __builtin_amdgcn_s_sleep(2);
  }
  if (d != 1u) {
    __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return -2;
  }
  return int(tk);
}

__device__ __forceinline__ unsigned xcc_id() {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  return xcc & 0xF;
}

}  // namespace
}  // namespace svm355
