// Device side of the native Cascade SVM (csrc/cascade): the gfx950 backend, the RCCL transport
// and the C ABI of the multi-GPU runs.
//
//   HipBackend     SV sets in HBM; assembly / packing are row-copy kernels on the rank's stream;
//                  every solve is the device trainer (MFMA / exact-integer RBF Gram + device SMO,
//                  warm start f from the resident Gram).  A caching allocator keeps the per-round
//                  sets from going back to hipMalloc / hipFree (hipFree synchronises the device).
//   RcclTransport  one communicator per GPU, collectives on the backend's stream (so they are
//                  ordered after the kernels that produced their buffers); every wait polls
//                  hipStreamQuery + ncclCommGetAsyncError against the WaitPolicy (abort token and
//                  deadline) instead of blocking in hipStreamSynchronize; abort() = ncclCommAbort.
//   C ABI          svmd_cascade_group_* : P thread-ranks over P GPUs of this process
//                                         (ncclCommInitAll) or a loopback rehearsal;
//                  svmd_cascade_rank_*  : one rank per process (ncclCommInitRank with an id the
//                                         launcher distributes, e.g. torchrun + a TCP store).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>

#include "cascade.h"
#include "cascade_capi.h"
#include "ctx.h"
#include "decomp.h"
#include "rccl_api.h"
#include "svm355_device.h"

namespace svm355 {
namespace {

inline const RcclApi& RC() { return rccl_checked(); }  // the explicitly loaded librccl (rccl_api.h)

// ------------------------------------------------------------------------------------- kernels
// One workgroup per row (grid-stride); rows of stored sets are 16-byte aligned (ld % 16 == 0), record
// rows (width ld + 3) are only 8-byte aligned.
__global__ __launch_bounds__(256) void assemble_set_kernel(const double* __restrict__ sX,
                                                           const int32_t* __restrict__ sy,
                                                           const double* __restrict__ sa,
                                                           const int64_t* __restrict__ sid,
                                                           const int64_t* __restrict__ idx, int64_t m, int64_t ld,
                                                           double* __restrict__ dX, int32_t* __restrict__ dy,
                                                           double* __restrict__ da, int64_t* __restrict__ did,
                                                           int zero_alpha) {
  for (int64_t i = blockIdx.x; i < m; i += gridDim.x) {
    const int64_t src = idx ? idx[i] : i;
    const double2* s = reinterpret_cast<const double2*>(sX + src * ld);
    double2* d = reinterpret_cast<double2*>(dX + i * ld);
    for (int64_t c = threadIdx.x; c < ld / 2; c += blockDim.x) d[c] = s[c];
    if (threadIdx.x == 0) {
      dy[i] = sy[src];
      da[i] = zero_alpha ? 0.0 : sa[src];
      did[i] = sid[src];
    }
  }
}

__global__ __launch_bounds__(256) void assemble_rec_kernel(const double* __restrict__ rec, int64_t w,
                                                           const int64_t* __restrict__ idx, int64_t m, int64_t ld,
                                                           double* __restrict__ dX, int32_t* __restrict__ dy,
                                                           double* __restrict__ da, int64_t* __restrict__ did,
                                                           int zero_alpha) {
  for (int64_t i = blockIdx.x; i < m; i += gridDim.x) {
    const double* r = rec + (idx ? idx[i] : i) * w;
    double* d = dX + i * ld;
    for (int64_t c = threadIdx.x; c < ld; c += blockDim.x) d[c] = r[c];
    if (threadIdx.x == 0) {
      dy[i] = int32_t(r[ld]);
      da[i] = zero_alpha ? 0.0 : r[ld + 1];
      did[i] = int64_t(r[ld + 2]);
    }
  }
}

__global__ __launch_bounds__(256) void pack_kernel(const double* __restrict__ X, const int32_t* __restrict__ y,
                                                   const double* __restrict__ a, const int64_t* __restrict__ id,
                                                   int64_t k, int64_t ld, double* __restrict__ rec) {
  const int64_t w = ld + 3;
  for (int64_t i = blockIdx.x; i < k; i += gridDim.x) {
    const double* s = X + i * ld;
    double* r = rec + i * w;
    for (int64_t c = threadIdx.x; c < ld; c += blockDim.x) r[c] = s[c];
    if (threadIdx.x == 0) {
      r[ld] = double(y[i]);
      r[ld + 1] = a[i];
      r[ld + 2] = double(id[i]);
    }
  }
}

__global__ void record_ids_kernel(const double* __restrict__ rec, int64_t k, int64_t w, int64_t ld,
                                  int64_t* __restrict__ out) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < k) out[i] = int64_t(rec[i * w + ld + 2]);
}

// SV extraction on the device (main3.cpp:297-304): the ascending indices i < k with a[i] > tol, to
// keep_d (device) and keep_h (pinned host), and their count to *count_h.  One 1024-thread workgroup
// walks the set in 1024-element chunks: per wave a ballot + prefix count, per chunk the wave totals.
__global__ __launch_bounds__(1024) void select_svs_kernel(const double* __restrict__ a, int64_t k, double tol,
                                                          int64_t* __restrict__ keep_d, int64_t* __restrict__ keep_h,
                                                          int64_t* __restrict__ count_h) {
  __shared__ int64_t wsum[16];
  __shared__ int64_t base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t c0 = 0; c0 < k; c0 += 1024) {
    const int64_t i = c0 + threadIdx.x;
    const bool f = i < k && a[i] > tol;
    const unsigned long long m = __ballot(f);
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int64_t off = base;
    for (int q = 0; q < w; ++q) off += wsum[q];
    if (f) {
      const int64_t pos = off + __popcll(m & ((1ull << lane) - 1ull));
      keep_d[pos] = i;
      keep_h[pos] = i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t t = 0;
      for (int q = 0; q < 16; ++q) t += wsum[q];
      base += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *count_h = base;
}

__global__ void coef_kernel(const double* __restrict__ a, const int32_t* __restrict__ y, int64_t nz,
                            double* __restrict__ coef) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < nz) coef[i] = a[i] * double(y[i]);
}

// One workgroup: f_i = s_i - y_i, then min f over I_high and max f over I_low (main3.cpp:107-142
// set definitions).  out = {b_high, b_low, #I_high, #I_low}.
__global__ __launch_bounds__(1024) void kkt_bounds_kernel(const double* __restrict__ s,
                                                          const int32_t* __restrict__ y,
                                                          const double* __restrict__ a, int64_t k, double C,
                                                          double eps, double* __restrict__ out) {
  double lo = __builtin_inf(), hi = -__builtin_inf();
  double nh = 0.0, nl = 0.0;
  for (int64_t i = threadIdx.x; i < k; i += blockDim.x) {
    const double f = s[i] - double(y[i]), ai = a[i];
    const bool pos = y[i] == 1;
    if ((pos && ai < C - eps) || (!pos && ai > eps)) {
      lo = fmin(lo, f);
      nh += 1.0;
    }
    if ((pos && ai > eps) || (!pos && ai < C - eps)) {
      hi = fmax(hi, f);
      nl += 1.0;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, off, kWave));
    hi = fmax(hi, __shfl_xor(hi, off, kWave));
    nh += __shfl_xor(nh, off, kWave);
    nl += __shfl_xor(nl, off, kWave);
  }
  __shared__ double part[16][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[w][0] = lo;
    part[w][1] = hi;
    part[w][2] = nh;
    part[w][3] = nl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < int(blockDim.x >> 6); ++q) {
      lo = fmin(lo, part[q][0]);
      hi = fmax(hi, part[q][1]);
      nh += part[q][2];
      nl += part[q][3];
    }
    out[0] = lo;
    out[1] = hi;
    out[2] = nh;
    out[3] = nl;
  }
}

unsigned row_grid(int64_t m) { return unsigned(std::min<int64_t>(m, 8192)); }

// --------------------------------------------------------------------------------- HipBackend
class HipBackend final : public Backend {
 public:
  explicit HipBackend(int device) : device_(device) {
    ctx_ = svmd_create(device);
    if (!ctx_) throw CascadeError(std::string("svmd_create: ") + svm_last_error());
    stream_ = static_cast<DeviceCtx*>(ctx_)->stream;
  }
  ~HipBackend() override {
    (void)hipSetDevice(device_);
    (void)hipStreamSynchronize(stream_);
    for (auto& kv : cache_) (void)hipFree(kv.second);
    for (auto& kv : live_) (void)hipFree(kv.first);  // includes the grow() scratch (allocator blocks)
    if (pinned_) (void)hipHostFree(pinned_);
    if (stage_ev_) (void)hipEventDestroy(stage_ev_);
    svmd_destroy(ctx_);
  }
  HipBackend(const HipBackend&) = delete;
  HipBackend& operator=(const HipBackend&) = delete;

  hipStream_t stream() const { return stream_; }
  DeviceCtx* device_ctx() const { return static_cast<DeviceCtx*>(ctx_); }
  int device() const { return device_; }
  const char* name() const override { return "hip"; }
  int64_t ld(int64_t d) const override { return svmd_padded_dim(d); }

  // Size-class caching allocator: blocks go back to a free list, never to hipFree, until the
  // backend is destroyed.  All users run on this backend's one stream, so reuse is stream-ordered.
  void* alloc(int64_t bytes) override {
    size_t cls = 256;
    while (cls < size_t(bytes)) cls <<= 1;
    auto it = cache_.find(cls);
    void* p = nullptr;
    if (it != cache_.end()) {
      p = it->second;
      cache_.erase(it);
    } else {
      hipcheck(hipSetDevice(device_), "hipSetDevice");
      if (hipMalloc(&p, cls) != hipSuccess) {
        release_cache();  // retry once with the cached blocks returned
        hipcheck(hipMalloc(&p, cls), "hipMalloc");
      }
    }
    live_[p] = cls;
    return p;
  }
  void free(void* p) override {
    auto it = live_.find(p);
    if (it == live_.end()) return;
    cache_.emplace(it->second, p);
    live_.erase(it);
  }
  void h2d(void* dst, const void* src, int64_t bytes) override {
    if (bytes > 0) check(svmd_memcpy_h2d(ctx_, dst, src, bytes), "svmd_memcpy_h2d");
  }
  void d2h(void* dst, const void* src, int64_t bytes) override {
    if (bytes > 0) check(svmd_memcpy_d2h(ctx_, dst, src, bytes), "svmd_memcpy_d2h");
  }
  void sync() override { check(svmd_synchronize(ctx_), "svmd_synchronize"); }
  void upload_rows(const void* X, bool u8, int64_t n, int64_t d, double* dst) override {
    if (!n) return;
    if (u8)
      check(svmd_upload_rows_u8(ctx_, static_cast<const uint8_t*>(X), n, d, dst, ld(d)), "svmd_upload_rows_u8");
    else
      check(svmd_upload_rows(ctx_, static_cast<const double*>(X), n, d, dst, ld(d)), "svmd_upload_rows");
  }
  void minmax(const double* X, int64_t n, int64_t d, double* mn, double* mx) override {
    if (n == 0) {  // an empty partition contributes the identities of min / max
      const std::vector<double> hi(size_t(d), __builtin_inf()), lo(size_t(d), -__builtin_inf());
      h2d(mn, hi.data(), d * 8);
      h2d(mx, lo.data(), d * 8);
      return;
    }
    check(svmd_minmax(ctx_, X, n, d, ld(d), mn, mx), "svmd_minmax");
  }
  void scale(double* X, int64_t n, int64_t d, const double* mn, const double* mx) override {
    check(svmd_preprocess(ctx_, X, n, d, ld(d), const_cast<double*>(mn), const_cast<double*>(mx), nullptr, 1),
          "svmd_preprocess");
  }
  void assemble(const Segment& s, int64_t ld, DSet& o, int64_t off) override {
    const int64_t m = s.rows();
    if (!m) return;
    const int64_t* idx = nullptr;
    if (s.idx) idx = s.idx_dev ? s.idx_dev : stage_idx(*s.idx);
    if (s.set) {
      hipLaunchKernelGGL(assemble_set_kernel, dim3(row_grid(m)), dim3(256), 0, stream_, s.set->X.as<double>(),
                         s.set->y.as<int32_t>(), s.set->a.as<double>(), s.set->id.as<int64_t>(), idx, m, ld,
                         o.X.as<double>() + off * ld, o.y.as<int32_t>() + off, o.a.as<double>() + off,
                         o.id.as<int64_t>() + off, int(s.zero_alpha));
    } else {
      hipLaunchKernelGGL(assemble_rec_kernel, dim3(row_grid(m)), dim3(256), 0, stream_, s.rec, ld + 3, idx, m, ld,
                         o.X.as<double>() + off * ld, o.y.as<int32_t>() + off, o.a.as<double>() + off,
                         o.id.as<int64_t>() + off, int(s.zero_alpha));
    }
    hipcheck(hipGetLastError(), "assemble kernel");
  }
  void pack(const DSet& S, int64_t ld, double* rec) override {
    if (!S.k) return;
    hipLaunchKernelGGL(pack_kernel, dim3(row_grid(S.k)), dim3(256), 0, stream_, S.X.as<double>(), S.y.as<int32_t>(),
                       S.a.as<double>(), S.id.as<int64_t>(), S.k, ld, rec);
    hipcheck(hipGetLastError(), "pack kernel");
  }
  void record_ids(const double* rec, int64_t k, int64_t ld, int64_t* ids) override {
    if (!k) return;
    grow(&ids_d_, &ids_cap_, size_t(k) * 8);
    hipLaunchKernelGGL(record_ids_kernel, dim3(unsigned((k + 255) / 256)), dim3(256), 0, stream_, rec, k, ld + 3, ld,
                       static_cast<int64_t*>(ids_d_));
    hipcheck(hipGetLastError(), "record_ids kernel");
    d2h(ids, ids_d_, k * 8);
  }
  void record_ids_batch(const std::vector<const double*>& recs, const std::vector<int64_t>& ks, int64_t ld,
                        const std::vector<int64_t*>& ids) override {
    int64_t tot = 0;
    for (int64_t k : ks) tot += k;
    if (!tot) return;
    grow(&ids_d_, &ids_cap_, size_t(tot) * 8);
    int64_t off = 0;
    for (size_t q = 0; q < recs.size(); ++q) {
      if (!ks[q]) continue;
      hipLaunchKernelGGL(record_ids_kernel, dim3(unsigned((ks[q] + 255) / 256)), dim3(256), 0, stream_, recs[q], ks[q],
                         ld + 3, ld, static_cast<int64_t*>(ids_d_) + off);
      hipcheck(hipGetLastError(), "record_ids kernel");
      off += ks[q];
    }
    std::vector<int64_t> all(static_cast<size_t>(tot));
    d2h(all.data(), ids_d_, tot * 8);  // one round trip for every source
    off = 0;
    for (size_t q = 0; q < recs.size(); ++q) {
      std::copy(all.begin() + off, all.begin() + off + ks[q], ids[q]);
      off += ks[q];
    }
  }
  // Device-side SV selection: the indices land in device memory (for the assembly kernel) and in
  // pinned host memory (for the host id mirror) with one synchronisation, instead of an alpha read
  // back, a host scan and an index upload.
  void select_svs(const DSet& S, double tol, std::vector<int64_t>* keep, const int64_t** keep_dev) override {
    keep->clear();
    *keep_dev = nullptr;
    if (!S.k) return;
    grow(&sel_d_, &sel_cap_, size_t(S.k) * 8);
    grow_pinned(size_t(S.k) * 8 + 64);
    auto* cnt = reinterpret_cast<int64_t*>(pinned_);
    auto* kh = cnt + 8;
    *cnt = -1;
    hipLaunchKernelGGL(select_svs_kernel, dim3(1), dim3(1024), 0, stream_, S.a.as<double>(), S.k, tol,
                       static_cast<int64_t*>(sel_d_), kh, cnt);
    hipcheck(hipGetLastError(), "select kernel");
    hipcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    if (*cnt < 0 || *cnt > S.k) throw CascadeError("device SV selection returned no count");
    keep->assign(kh, kh + *cnt);
    *keep_dev = static_cast<const int64_t*>(sel_d_);
  }
  SolveStats solve(DSet& S, int64_t d, const svm_params& p, const double* mn_h, const double* mx_h, int solver,
                   int64_t) override {
    if (solver == 1) {  // the decomposition solver keeps no Gram: nothing to size or hand back
      SolveStats st;
      if (solo([&] { return solve_decomp(S, d, p, mn_h, mx_h, &st); })) return st;
    }
    if (!(serial_ && release_gram_)) return solo([&] { return solve_impl(S, d, p, mn_h, mx_h); });
    // Large-n rehearsals of P ranks on one GPU (SVM355_CASCADE_RELEASE_GRAM=1 with serial solves):
    // P resident Grams do not fit together, so each solve's Gram is sized before its timed region
    // (the grow-only buffer a rank keeps on its own GPU) and handed back after it, under the lock.
    return solo([&] { return solve_impl(S, d, p, mn_h, mx_h); },
                [&] { (void)svmd_reserve_gram(ctx_, S.k); },
                [&] { check(svmd_release_cache(ctx_), "svmd_release_cache"); });
  }
  bool warm_start_converged(DSet& S, int64_t nz, int64_t d, const svm_params& p, const double* mn_h,
                            const double* mx_h) override {
    return solo([&] { return kkt_check(S, nz, d, p, mn_h, mx_h); });
  }
  double take_solo_ms() override {
    if (!solo_any_) return -1.0;
    const double v = solo_acc_;
    solo_acc_ = 0.0;
    solo_any_ = false;
    return v;
  }
  void trace_push(const char* name) override { svmd_trace_push(name); }
  void trace_pop() override { svmd_trace_pop(); }

 private:
  // SVM355_CASCADE_SERIAL_SOLVES=1: solves (and skip checks) of all ranks of this process take one
  // lock, and each is timed from an idle stream to its completion -- the device time the solve
  // would take on a GPU of its own (one-GPU rehearsals of P ranks; bench.py's critical path).
  static std::mutex& solo_mutex() {
    static std::mutex m;
    return m;
  }
  // pre / post run under the lock, outside the timed region.
  template <class F, class Pre = void (*)(), class Post = void (*)()>
  decltype(std::declval<F&>()()) solo(F&& f, Pre&& pre = [] {}, Post&& post = [] {}) {
    if (!serial_) return f();
    std::lock_guard<std::mutex> lk(solo_mutex());
    pre();
    sync();
    const auto t0 = std::chrono::steady_clock::now();
    auto r = f();
    sync();
    solo_acc_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    solo_any_ = true;
    post();
    return r;
  }
  // Warm-started working-set decomposition (decomp.hip) on the set's scaled rows: quantised with the
  // global statistics into the exact-integer plan, f = K (alpha y) - y from the warm alphas by the
  // solver's GEMV, then the decomposition to the reference's stop test.  False (nothing done) when
  // the set admits no exact-integer plan or has fewer than 2 rows: the pairwise solve runs instead.
  bool solve_decomp(DSet& S, int64_t d, const svm_params& p, const double* mn_h, const double* mx_h,
                    SolveStats* out) {
    if (S.k < 2 || !mn_h || !mx_h) return false;
    svm_result r{};
    int64_t st[kDecompStats] = {};
    bool used = false;
    double prep = 0.0;
    DecompOpts o;
    o.warm = true;
    // A/B probe: SVM355_DECOMP_CASCADE_START=cold starts every solve from alpha = 0 (the same local
    // optimum, another path); the reference warm-starts (mpi_svm_main3.cpp:169-186)
    if (const char* cs = getenv("SVM355_DECOMP_CASCADE_START")) o.warm = strcmp(cs, "cold") != 0;
    check(decomp_fit_rows(device_ctx(), S.X.as<double>(), S.k, ld(d), d, mn_h, mx_h, S.y.as<int32_t>(),
                          S.a.as<double>(), p, 1024, &r, st, &used, &prep, o),
          "decomposition SMO");
    if (!used) return false;
    *out = SolveStats{r.iterations, r.b, r.stop_reason, prep};
    out->solver = 1;
    out->outer = st[0];
    return true;
  }
  SolveStats solve_impl(DSet& S, int64_t d, const svm_params& p, const double* mn_h, const double* mx_h) {
    const int64_t ldd = ld(d);
    grow(&sqn_, &sqn_cap_, size_t(S.k) * 8);
    auto* sqn = static_cast<double*>(sqn_);
    check(svmd_row_norms(ctx_, S.X.as<double>(), S.k, d, ldd, sqn), "svmd_row_norms");
    svm_result r{};
    svmd_timing tm{};
    int32_t used = 0;
    // A partition whose k x k Gram does not fit (large-n cascades; ranks sharing one GPU in a
    // loopback rehearsal) is solved on the HBM row cache instead: the same exact-integer kernel
    // values, computed on demand (rowcache.hip / smo.hip's persistent row-cache solver).
    // SVM355_CASCADE_GRAM=rows forces that path (tests).
    const char* gm = getenv("SVM355_CASCADE_GRAM");
    int rc = SVM_ERR_OOM;
    if (!(gm && !strcmp(gm, "rows")))
      rc = svmd_train_q(ctx_, S.X.as<double>(), sqn, S.k, ldd, ldd, S.y.as<int32_t>(), S.a.as<double>(), 1, &p, &r,
                        nullptr, 0, &tm, mn_h, mx_h, d, 0, &used);
    const bool on_rows = rc == SVM_ERR_OOM;
    if (on_rows) {
      release_cache();  // unused blocks of this backend's set allocator, then the context's Gram
      check(svmd_release_cache(ctx_), "svmd_release_cache");
      rc = svmd_train_rows(ctx_, S.X.as<double>(), sqn, S.k, ldd, d, S.y.as<int32_t>(), S.a.as<double>(), 1, &p, &r,
                           mn_h, mx_h, 0, 0, &used, nullptr, 0);
    }
    check(rc, "svmd_train");
    return SolveStats{r.iterations, r.b, r.stop_reason, tm.gram_ms, on_rows};
  }
  // f from the cross-kernel K(S, S[0:nz]): the exact-integer block (int8 MFMA, the very values of
  // the Gram the solve would build) for pixel data, else the MFMA f64 decision path, whose values
  // agree with the Gram's to a few ulps, so f agrees to ~1e-9 here (nz <= a few thousand,
  // alpha <= C); a 1e-7 margin on the stop test covers either.
  // The check is an optimisation only: a failure of its own (e.g. its k x nz workspace does not fit
  // next to a large partition) answers "not converged" and the normal solve runs.
  bool kkt_check(DSet& S, int64_t nz, int64_t d, const svm_params& p, const double* mn_h, const double* mx_h) {
    try {
      return kkt_check_impl(S, nz, d, p, mn_h, mx_h);
    } catch (const CascadeError&) {
      (void)hipGetLastError();  // clear a sticky launch / allocation error of the failed attempt
      return false;
    }
  }
  bool kkt_check_impl(DSet& S, int64_t nz, int64_t d, const svm_params& p, const double* mn_h, const double* mx_h) {
    const char* e = getenv("SVM355_CASCADE_SKIP");  // =0 disables the check (A/B runs, tests)
    if ((e && atoi(e) == 0) || nz <= 0 || nz > S.k) return false;
    const int64_t ldd = ld(d), k = S.k;
    grow(&sqn_, &sqn_cap_, size_t(k) * 8);
    grow(&kkt_, &kkt_cap_, size_t(nz + k + 8) * 8);
    auto* sqn = static_cast<double*>(sqn_);
    auto* coef = static_cast<double*>(kkt_);
    double* sum = coef + nz;
    double* res = sum + k;
    check(svmd_row_norms(ctx_, S.X.as<double>(), k, d, ldd, sqn), "svmd_row_norms");
    hipLaunchKernelGGL(coef_kernel, dim3(unsigned((nz + 255) / 256)), dim3(256), 0, stream_, S.a.as<double>(),
                       S.y.as<int32_t>(), nz, coef);
    hipcheck(hipGetLastError(), "coef kernel");
    int32_t used_int = 0;
    const char* ki = getenv("SVM355_CASCADE_SKIP_INT");  // =0: always the f64 cross-kernel (A/B)
    if (!(ki && atoi(ki) == 0) && mn_h && mx_h)
      check(svmd_decision_int(ctx_, S.X.as<double>(), k, ldd, d, mn_h, mx_h, coef, nz, p.gamma, sum, &used_int),
            "svmd_decision_int");
    if (!used_int)
      check(svmd_decision(ctx_, S.X.as<double>(), sqn, coef, nz, ldd, S.X.as<double>(), sqn, k, ldd, ldd, p.gamma,
                          0.0, sum),
            "svmd_decision");
    hipLaunchKernelGGL(kkt_bounds_kernel, dim3(1), dim3(1024), 0, stream_, sum, S.y.as<int32_t>(), S.a.as<double>(), k,
                       p.C, p.eps, res);
    hipcheck(hipGetLastError(), "kkt kernel");
    double h[4];
    d2h(h, res, sizeof(h));
    if (h[2] < 1 || h[3] < 1) return false;  // no candidate: the solve reports it
    constexpr double kMargin = 1e-7;
    return h[1] <= h[0] + 2.0 * p.tau - kMargin;
  }
  static void check(int rc, const char* what) {
    if (rc != SVM_OK) throw CascadeError(std::string(what) + ": " + svm_last_error());
  }
  static void hipcheck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw CascadeError(std::string(what) + ": " + hipGetErrorString(e));
  }
  // Grow-only scratch through the size-class caching allocator: the old block goes back to the
  // cache (reuse is stream-ordered: every user runs on this backend's one stream), no sync, no
  // hipFree.
  void grow(void** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return;
    if (*p) free(*p);
    *p = nullptr;
    *cap = 0;
    const size_t sz = std::max<size_t>(bytes, 4096) * 2;
    *p = alloc(int64_t(sz));
    *cap = sz;
  }
  // Pinned host staging area (grow-only; waits for the copy still reading it before it is reused).
  void grow_pinned(size_t bytes) {
    wait_staged();
    if (bytes <= pinned_cap_) return;
    if (pinned_) {
      hipcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");  // a kernel may still write it
      hipcheck(hipHostFree(pinned_), "hipHostFree");
    }
    pinned_ = nullptr;
    pinned_cap_ = 0;
    const size_t sz = std::max<size_t>(bytes, 1 << 16) * 2;
    hipcheck(hipHostMalloc(&pinned_, sz, hipHostMallocDefault), "hipHostMalloc");
    pinned_cap_ = sz;
  }
  void wait_staged() {
    if (staged_) {
      hipcheck(hipEventSynchronize(stage_ev_), "hipEventSynchronize");
      staged_ = false;
    }
  }
  // Index list -> device through the pinned area with an asynchronous copy: the caller's vector may
  // go away at once, and the next staging waits only for this copy (not for the whole stream).
  const int64_t* stage_idx(const std::vector<int64_t>& v) {
    grow(&idx_, &idx_cap_, v.size() * 8);
    grow_pinned(v.size() * 8);
    std::memcpy(pinned_, v.data(), v.size() * 8);
    hipcheck(hipMemcpyAsync(idx_, pinned_, v.size() * 8, hipMemcpyHostToDevice, stream_), "hipMemcpyAsync idx");
    if (!stage_ev_) hipcheck(hipEventCreateWithFlags(&stage_ev_, hipEventDisableTiming), "hipEventCreate");
    hipcheck(hipEventRecord(stage_ev_, stream_), "hipEventRecord");
    staged_ = true;
    return static_cast<const int64_t*>(idx_);
  }
  void release_cache() {
    hipcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    for (auto& kv : cache_) (void)hipFree(kv.second);
    cache_.clear();
  }

  int device_;
  void* ctx_ = nullptr;
  hipStream_t stream_ = nullptr;
  std::multimap<size_t, void*> cache_;
  std::map<void*, size_t> live_;
  void *idx_ = nullptr, *ids_d_ = nullptr, *sqn_ = nullptr, *kkt_ = nullptr, *sel_d_ = nullptr;
  size_t idx_cap_ = 0, ids_cap_ = 0, sqn_cap_ = 0, kkt_cap_ = 0, sel_cap_ = 0;
  void* pinned_ = nullptr;  // host staging (index uploads, device SV selection results)
  size_t pinned_cap_ = 0;
  hipEvent_t stage_ev_ = nullptr;
  bool staged_ = false;
  const bool serial_ = [] {
    const char* v = getenv("SVM355_CASCADE_SERIAL_SOLVES");
    return v && atoi(v) != 0;
  }();
  const bool release_gram_ = [] {
    const char* v = getenv("SVM355_CASCADE_RELEASE_GRAM");
    return v && atoi(v) != 0;
  }();
  double solo_acc_ = 0.0;
  bool solo_any_ = false;
};

// ------------------------------------------------------------------------------ RcclTransport
#define NCCLT(expr)                                                                                 \
  do {                                                                                              \
    const ncclResult_t r_ = (expr);                                                                 \
    if (r_ != ncclSuccess) throw TransportError(std::string(#expr) + ": " + RC().GetErrorString(r_)); \
  } while (0)
#define HIPT(expr)                                                                                    \
  do {                                                                                                \
    const hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) throw TransportError(std::string(#expr) + ": " + hipGetErrorString(e_));     \
  } while (0)

class RcclTransport final : public Transport {
 public:
  RcclTransport(ncclComm_t comm, int device, hipStream_t stream, WaitPolicy wp)
      : comm_(comm), device_(device), stream_(stream), wp_(std::move(wp)) {
    HIPT(hipSetDevice(device_));
    NCCLT(RC().CommUserRank(comm_, &rank_));
    NCCLT(RC().CommCount(comm_, &world_));
    HIPT(hipMalloc(&scratch_, size_t(64 + world_) * 8));
    HIPT(hipHostMalloc(&pinned_, size_t(64 + world_) * 8, hipHostMallocDefault));
  }
  ~RcclTransport() override {
    (void)hipSetDevice(device_);
    (void)hipStreamSynchronize(stream_);
    if (scratch_) (void)hipFree(scratch_);
    if (pinned_) (void)hipHostFree(pinned_);
  }
  bool aborted() const { return aborted_; }
  void set_policy(WaitPolicy wp) { wp_ = std::move(wp); }  // per fit: a fresh abort token
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  const char* name() const override { return "rccl"; }

  int64_t bcast_i64(int64_t v, int root) override {
    static const bool prof = [] {
      const char* e = getenv("SVM355_CASCADE_PROFILE");
      return e && atoi(e) >= 3;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t q0 = prof ? hipStreamQuery(stream_) : hipSuccess;
    pinned_[0] = v;
    HIPT(hipMemcpyAsync(scratch_, pinned_, 8, hipMemcpyHostToDevice, stream_));
    const auto t1 = std::chrono::steady_clock::now();
    NCCLT(RC().Broadcast(scratch_, scratch_, 1, ncclInt64, root, comm_, stream_));
    const auto t2 = std::chrono::steady_clock::now();
    HIPT(hipMemcpyAsync(pinned_ + 1, scratch_, 8, hipMemcpyDeviceToHost, stream_));
    wait("ncclBroadcast(i64)");
    if (prof) {
      auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      fprintf(stderr, "[rccl bcast_i64] stream idle at entry %d | h2d enqueue %.3f | bcast enqueue %.3f | rest %.3f ms\n",
              int(q0 == hipSuccess), ms(t0, t1), ms(t1, t2), ms(t2, std::chrono::steady_clock::now()));
    }
    return pinned_[1];
  }
  std::vector<int64_t> allgather_i64(int64_t v) override {
    pinned_[0] = v;
    HIPT(hipMemcpyAsync(scratch_, pinned_, 8, hipMemcpyHostToDevice, stream_));
    NCCLT(RC().AllGather(scratch_, scratch_ + 1, 1, ncclInt64, comm_, stream_));
    HIPT(hipMemcpyAsync(pinned_ + 1, scratch_ + 1, size_t(world_) * 8, hipMemcpyDeviceToHost, stream_));
    wait("ncclAllGather(i64)");
    return std::vector<int64_t>(pinned_ + 1, pinned_ + 1 + world_);
  }
  void allreduce_min(double* buf, int64_t n) override {
    NCCLT(RC().AllReduce(buf, buf, size_t(n), ncclFloat64, ncclMin, comm_, stream_));
    wait("ncclAllReduce(min)");
  }
  void allreduce_max(double* buf, int64_t n) override {
    NCCLT(RC().AllReduce(buf, buf, size_t(n), ncclFloat64, ncclMax, comm_, stream_));
    wait("ncclAllReduce(max)");
  }
  void bcast(void* buf, int64_t bytes, int root) override {
    if (bytes <= 0) return;
    NCCLT(RC().Broadcast(buf, buf, size_t(bytes), ncclUint8, root, comm_, stream_));
    wait("ncclBroadcast");
  }
  void gather(const void* send, int64_t bytes, void* recv, int root) override {
    if (bytes <= 0) return;
    NCCLT(RC().Gather(send, recv, size_t(bytes), ncclUint8, root, comm_, stream_));
    wait("ncclGather");
  }
  void allgather(const void* send, int64_t bytes, void* recv) override {
    if (bytes <= 0) return;
    NCCLT(RC().AllGather(send, recv, size_t(bytes), ncclUint8, comm_, stream_));
    wait("ncclAllGather");
  }
  void allgather_async(const void* send, int64_t bytes, void* recv) override {
    if (bytes > 0) NCCLT(RC().AllGather(send, recv, size_t(bytes), ncclUint8, comm_, stream_));
  }
  bool stream_wait(const char* what) override {
    wait(what);
    return true;
  }
  bool event_wait(void* event, const char* what) override {
    wait(what, static_cast<hipEvent_t>(event));
    return true;
  }
  void send_i64(int64_t v, int peer) override {
    pinned_[2] = v;
    HIPT(hipMemcpyAsync(scratch_ + 2, pinned_ + 2, 8, hipMemcpyHostToDevice, stream_));
    NCCLT(RC().Send(scratch_ + 2, 1, ncclInt64, peer, comm_, stream_));
    wait("ncclSend(i64)");
  }
  int64_t recv_i64(int peer) override {
    NCCLT(RC().Recv(scratch_ + 3, 1, ncclInt64, peer, comm_, stream_));
    HIPT(hipMemcpyAsync(pinned_ + 3, scratch_ + 3, 8, hipMemcpyDeviceToHost, stream_));
    wait("ncclRecv(i64)");
    return pinned_[3];
  }
  void send(const void* buf, int64_t bytes, int peer) override {
    if (bytes <= 0) return;
    NCCLT(RC().Send(buf, size_t(bytes), ncclUint8, peer, comm_, stream_));
    wait("ncclSend");
  }
  void recv(void* buf, int64_t bytes, int peer) override {
    if (bytes <= 0) return;
    NCCLT(RC().Recv(buf, size_t(bytes), ncclUint8, peer, comm_, stream_));
    wait("ncclRecv");
  }
  void barrier() override {
    NCCLT(RC().AllReduce(scratch_ + 4, scratch_ + 4, 1, ncclInt64, ncclSum, comm_, stream_));
    wait("ncclAllReduce(barrier)");
  }
  void abort() override {
    if (aborted_ || !comm_) return;
    aborted_ = true;
    (void)RC().CommAbort(comm_);  // frees the communicator; in-flight kernels are torn down
  }

 private:
  // Poll instead of hipStreamSynchronize: a peer that never arrives must not hang this thread.
  void wait(const char* what, hipEvent_t event = nullptr) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
      const hipError_t e = event ? hipEventQuery(event) : hipStreamQuery(stream_);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) throw TransportError(std::string(what) + ": " + hipGetErrorString(e));
      ncclResult_t ae = ncclSuccess;
      if (RC().CommGetAsyncError(comm_, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
        throw TransportError(std::string(what) + ": " + RC().GetErrorString(ae));
      wp_.check(t0, what);
      if (spin < 2000)
        std::this_thread::yield();
      else
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  ncclComm_t comm_;
  int device_, rank_ = 0, world_ = 1;
  hipStream_t stream_;
  WaitPolicy wp_;
  int64_t* scratch_ = nullptr;
  int64_t* pinned_ = nullptr;
  bool aborted_ = false;
};

double timeout_or_default(double s) { return s > 0 ? s : 600.0; }

// ---- RCCL runtime identity.  The entry points come from the librccl loaded explicitly by
// rccl_api.h (the one the headers belong to; inside a PyTorch process a -lrccl link would bind to
// torch's bundled, older copy instead).  The version check stays as a guard for SVM355_RCCL_LIB
// overrides: a runtime of the header's major version and at least kMinRcclCode is accepted, an older
// minor than the header's is reported as a skew, and the preflight (exercise.cpp) checks every op on
// the live communicators anyway.
constexpr int kMinRcclCode = 21200;
struct RcclInfo {
  int header = NCCL_VERSION_CODE;
  int runtime = 0;
  std::string path;
};
const RcclInfo& rccl_info() {
  static const RcclInfo info = [] {
    RcclInfo r;
    const RcclApi& a = rccl();
    if (!a.ok() || a.GetVersion(&r.runtime) != ncclSuccess) r.runtime = 0;
    r.path = a.ok() ? a.path : a.error;
    return r;
  }();
  return info;
}
void require_rccl_runtime() {
  const RcclInfo& i = rccl_info();
  if (i.runtime / 10000 != NCCL_MAJOR || i.runtime < kMinRcclCode)
    throw CascadeError("RCCL runtime " + std::to_string(i.runtime) + " (" + i.path + ") is not usable: need major " +
                       std::to_string(NCCL_MAJOR) + " and at least " + std::to_string(kMinRcclCode) +
                       " (built against " + std::to_string(i.header) + ")");
}

// Preflight: the driver's whole op set over the live communicators (SVM355_RCCL_PREFLIGHT=0 skips it).
constexpr double kPreflightTimeout = 20.0;
constexpr int64_t kPreflightBytes = 1 << 20;
bool preflight_enabled() {
  const char* e = getenv("SVM355_RCCL_PREFLIGHT");
  return !(e && atoi(e) == 0);
}

// ------------------------------------------------------------------------- thread-rank group
struct Group {
  int world = 0;
  bool rccl = false;
  bool broken = false;
  double timeout_s = 600.0;
  std::vector<int> devices;
  std::vector<std::unique_ptr<HipBackend>> be;
  std::vector<ncclComm_t> comms;
  std::vector<std::unique_ptr<RcclTransport>> rtr;  // persistent (pinned / device scratch)
  std::unique_ptr<RankPool> pool;                   // one persistent host thread per rank
  std::mutex mu;  // one fit at a time
  // loopback rehearsal with SVM355_CASCADE_SERIAL_SOLVES=1: the distributed decomposition's per-rank
  // solo segment times (DecompSolo) and their summary (svmd_cascade_group_decomp_solo)
  std::mutex solo_mu;
  std::vector<double> solo_report;
  std::vector<double> host_wait_ms;  // the last distributed decomposition fit's per-rank host wait
};

// ----------------------------------------------------------------------------- process rank
// tr: RCCL over the rank's communicator, or (svmd_cascade_rank_create_hostcomm) the caller's host
// collectives with device buffers staged through host memory -- the per-process launch rehearsed with
// several processes on one GPU, where RCCL refuses to run.
struct ProcRank {
  int device = 0;
  bool broken = false;
  double timeout_s = 600.0;
  std::unique_ptr<HipBackend> be;
  ncclComm_t comm = nullptr;
  std::unique_ptr<Transport> tr;
  RcclTransport* rccl = nullptr;  // tr when it is RCCL (deadline / abort policy per call)
  double host_wait_ms = 0.0;       // the last distributed decomposition fit's host wait
  void set_policy(WaitPolicy wp) {
    if (rccl) rccl->set_policy(std::move(wp));
  }
};

// Runs `script` (exercise.cpp) on every rank of a group; "" on success, else the first error (the
// group is then broken: its communicators were aborted).
std::string group_exercise(Group& g, const std::string& script, double timeout_s) {
  const int P = g.world;
  auto token = std::make_shared<AbortToken>();
  const WaitPolicy wp{token, timeout_s};
  std::vector<Transport*> tr(static_cast<size_t>(P));
  std::vector<std::unique_ptr<LoopbackTransport>> ltr;
  std::shared_ptr<LoopbackGroup> lg = g.rccl ? nullptr : std::make_shared<LoopbackGroup>(P, wp);
  for (int r = 0; r < P; ++r) {
    if (g.rccl) {
      g.rtr[size_t(r)]->set_policy(wp);
      tr[size_t(r)] = g.rtr[size_t(r)].get();
    } else {
      ltr.push_back(std::make_unique<LoopbackTransport>(lg, r, g.be[size_t(r)].get()));
      tr[size_t(r)] = ltr.back().get();
    }
  }
  try {
    g.pool->run(
        token,
        [&](int r) {
          if (hipSetDevice(g.devices[size_t(r)]) != hipSuccess) throw CascadeError("hipSetDevice failed");
          exercise_transport(*tr[size_t(r)], *g.be[size_t(r)], script);
        },
        [&](int r) {
          (void)hipSetDevice(g.devices[size_t(r)]);
          tr[size_t(r)]->abort();
        });
  } catch (const std::exception& e) {
    if (g.rccl) g.broken = true;
    return e.what();
  }
  return "";
}

// One rank of the distributed decomposition SMO (decomp.hip): the rank's GPU gets all n rows and
// labels and runs the solve over its block range with the candidate records all-gathered through `tr`
// (null: one GPU).  u8: uint8 pixel rows (quantised on the device: exact-integer kernel values); else
// FP64 rows (n x d, the reference's format, mpi_svm_main2.cpp:316-402 / mpi_svm_main3.cpp:433-518):
// min-max scaled on the device, then the exact-integer plan when their values admit one, FP64-MFMA kernel
// values otherwise (real-valued data; decomp_fit_rows).  alpha_out (host, n doubles) may be null.
// uint8 rows whose column ranges admit no exact-integer plan within the int8 kernels' 4,096 columns (wide
// rows with many distinct ranges) are solved as FP64 rows: `widen` re-runs the rank with the host bytes
// widened to doubles on upload -- the single-GPU SVC's fallback (svc.py _fit_cuda_u8 ->
// train_decomp_rows), taken by every rank alike (the plan is a function of the global min / max).
void decomp_on_rank(HipBackend& be, Transport* tr, const void* Xv, bool u8, const int32_t* y, int64_t n, int64_t d,
                    const svm_params& p, int q, double* alpha_out, svm_result* r, int64_t* stats, double* ms_out,
                    double* mm_out, DecompSolo* solo = nullptr, double* host_wait_ms = nullptr, bool widen = false) {
  const auto t0 = std::chrono::steady_clock::now();
  auto check = [](int rc, const char* what) {
    if (rc != SVM_OK) throw CascadeError(std::string(what) + ": " + svm_last_error());
  };
  DeviceCtx* ctx = be.device_ctx();
  const int world = tr ? tr->world() : 1, rank = tr ? tr->rank() : 0;
  // Each GPU copies 1/world of the rows from the host over its own link and the rows are all-gathered
  // over xGMI (in place), instead of every GPU pulling all n rows through the host: world concurrent
  // pageable copies of the whole set would be staged through host memory world times.
  const bool u8dev = u8 && !widen;  // the device rows are the host's bytes
  const int64_t ld = u8dev ? d : svmd_padded_dim(d), esz = u8dev ? 1 : 8;
  const int64_t rows_per = (n + world - 1) / world, chunk = rows_per * ld * esz;
  auto* Xd = static_cast<char*>(be.alloc(chunk * world));
  auto* yd = static_cast<int32_t*>(be.alloc(n * 4));
  auto* ad = static_cast<double*>(be.alloc(n * 8));
  auto* mm = static_cast<double*>(be.alloc(2 * d * 8));
  struct Free {
    HipBackend& b;
    std::vector<void*> ptrs;
    ~Free() {
      for (void* q : ptrs) b.free(q);
    }
  } fr{be, {Xd, yd, ad, mm}};
  const int64_t r0 = std::min<int64_t>(n, rank * rows_per), r1 = std::min<int64_t>(n, r0 + rows_per);
  const char* Xh = static_cast<const char*>(Xv);
  auto upload = [&](int64_t a0, int64_t a1, char* dst) {  // host rows [a0, a1) to the device (FP64: padded to ld)
    if (a1 <= a0) return;
    if (u8dev) {
      be.h2d(dst, Xh + a0 * d, (a1 - a0) * d);
    } else if (widen) {  // the bytes widened to doubles on the device (svmd_upload_rows_u8)
      be.upload_rows(Xh + a0 * d, true, a1 - a0, d, reinterpret_cast<double*>(dst));
    } else {
      be.upload_rows(Xh + a0 * d * 8, false, a1 - a0, d, reinterpret_cast<double*>(dst));
    }
  };
  if (world > 1) {
    upload(r0, r1, Xd + rank * chunk);
    tr->allgather(Xd + rank * chunk, chunk, Xd);  // rank r's slice at r * chunk = row r * rows_per
  } else {
    upload(0, n, Xd);
  }
  be.h2d(yd, y, n * 4);
  if (u8dev)
    check(svmd_minmax_u8(ctx, reinterpret_cast<uint8_t*>(Xd), n, d, mm, mm + d), "svmd_minmax_u8");
  else  // the single-GPU SVC's scaling (svmd_preprocess: column min / max, then the rows scaled in place)
    check(svmd_preprocess(ctx, reinterpret_cast<double*>(Xd), n, d, ld, mm, mm + d, nullptr, 0), "svmd_preprocess");
  std::vector<double> mmh(size_t(2 * d));
  be.d2h(mmh.data(), mm, 2 * d * 8);
  if (mm_out) std::memcpy(mm_out, mmh.data(), size_t(2 * d) * 8);
  // RCCL: the all-gather is only enqueued; the solver's one host wait per outer iteration (after the
  // working-set build that reads the gathered candidates) polls under the transport's deadline
  DecompOpts o;
  o.world = world;
  o.rank = rank;
  o.solo = solo;
  o.host_wait_ms = host_wait_ms;
  if (tr)
    o.allgather = {[tr](const void* send, int64_t bytes, void* recv) { tr->allgather_async(send, bytes, recv); },
                   [tr](void* ev) { return tr->event_wait(ev, "decomposition SMO: a batch of outer iterations"); }};
  bool used = false;
  double prep = 0.0;
  svm_result res{};
  // fault injection (tests): SVM355_DECOMP_FAIL_RANK / _OUTER make that rank fail at that outer
  // iteration inside the solve (run_decomp) while the others wait in their candidate all-gather; the
  // group's abort must end every rank with an error, not a hang
  if (u8dev)
    check(decomp_fit_u8(ctx, reinterpret_cast<uint8_t*>(Xd), n, d, mmh.data(), mmh.data() + d, yd, ad, p, q, &res,
                        stats, &used, &prep, o),
          "decomposition SMO");
  else
    check(decomp_fit_rows(ctx, reinterpret_cast<double*>(Xd), n, ld, d, mmh.data(), mmh.data() + d, yd, ad, p, q, &res,
                          stats, &used, &prep, o),
          "decomposition SMO");
  if (!used && u8dev && n >= 2 && n <= (int64_t(1) << 31) - 2) {
    // no exact-integer plan for these bytes (more than 4,096 int8 columns after grouping): FP64 rows
    for (void* b : fr.ptrs) be.free(b);  // the byte rows' buffers, before the FP64 rows are allocated
    fr.ptrs.clear();
    decomp_on_rank(be, tr, Xv, u8, y, n, d, p, q, alpha_out, r, stats, nullptr, mm_out, solo, host_wait_ms, true);
    if (ms_out) *ms_out = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return;
  }
  if (!used)
    throw CascadeError("decomposition SMO: n = " + std::to_string(n) + " is outside 2 .. 2^31 - 2, or the "
                       "FP64-row solve's workspace (n / world x 1,024 doubles per GPU) does not fit");
  if (alpha_out) be.d2h(alpha_out, ad, n * 8);
  be.sync();
  if (r) *r = res;
  if (ms_out) *ms_out = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace
}  // namespace svm355

using namespace svm355;

extern "C" {

SVM_API int svmd_rccl_info(int32_t* header_code, int32_t* runtime_code, char* path, int64_t cap) {
  const RcclInfo& i = rccl_info();
  if (header_code) *header_code = i.header;
  if (runtime_code) *runtime_code = i.runtime;
  if (path && cap > 0) {
    std::strncpy(path, i.path.c_str(), size_t(cap) - 1);
    path[cap - 1] = 0;
  }
  return SVM_OK;
}

SVM_API int svmd_cascade_group_exercise(void* h, const char* script, double timeout_s) {
  auto* g = static_cast<Group*>(h);
  if (!g || !script) {
    set_error("svmd_cascade_group_exercise: bad arguments");
    return SVM_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(g->mu);
  if (g->broken) {
    set_error("svmd_cascade_group_exercise: the group's communicators were aborted by an earlier failure");
    return SVM_ERR_ARG;
  }
  const std::string err = group_exercise(*g, script, timeout_s > 0 ? timeout_s : kPreflightTimeout);
  if (!err.empty()) {
    set_error("%s", err.c_str());
    return SVM_ERR_DEVICE;
  }
  return SVM_OK;
}

SVM_API int svmd_cascade_group_broken(void* h) { return h && static_cast<Group*>(h)->broken ? 1 : 0; }

SVM_API void* svmd_cascade_group_create(int32_t world, const char* transport, double comm_timeout_s) {
  try {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    if (world < 1) throw CascadeError("world must be >= 1");
    if (ndev < 1) throw CascadeError("no HIP device visible");
    std::string tr = transport ? transport : "auto";
    if (tr == "auto") tr = world <= ndev ? "rccl" : "loopback";
    if (tr != "rccl" && tr != "loopback") throw CascadeError("transport must be auto, rccl or loopback");
    if (tr == "rccl" && world > ndev)
      throw CascadeError("rccl transport needs one GPU per rank (" + std::to_string(world) + " ranks, " +
                         std::to_string(ndev) + " GPUs visible)");
    auto g = std::make_unique<Group>();
    g->world = world;
    g->rccl = tr == "rccl";
    g->timeout_s = timeout_or_default(comm_timeout_s);
    for (int r = 0; r < world; ++r) {
      g->devices.push_back(g->rccl ? r : r % ndev);
      g->be.push_back(std::make_unique<HipBackend>(g->devices.back()));
    }
    if (g->rccl) {
      g->comms.resize(size_t(world));
      const ncclResult_t rc = RC().CommInitAll(g->comms.data(), world, g->devices.data());
      if (rc != ncclSuccess) throw CascadeError(std::string("ncclCommInitAll: ") + RC().GetErrorString(rc));
      for (int r = 0; r < world; ++r)
        g->rtr.push_back(std::make_unique<RcclTransport>(g->comms[size_t(r)], g->devices[size_t(r)],
                                                         g->be[size_t(r)]->stream(), WaitPolicy{}));
    }
    g->pool = std::make_unique<RankPool>(world);
    if (g->rccl) {
      require_rccl_runtime();
      if (preflight_enabled()) {
        const std::string err = group_exercise(*g, preflight_script(world, kPreflightBytes), kPreflightTimeout);
        if (!err.empty()) {
          Group* raw = g.release();
          svmd_cascade_group_destroy(raw);  // communicators were aborted by the failed exercise
          throw CascadeError("RCCL preflight failed: " + err);
        }
      }
    }
    return g.release();
  } catch (const std::exception& e) {
    set_error("svmd_cascade_group_create: %s", e.what());
    return nullptr;
  }
}

SVM_API void svmd_cascade_group_destroy(void* h) {
  auto* g = static_cast<Group*>(h);
  if (!g) return;
  g->pool.reset();
  g->rtr.clear();
  if (!g->broken)
    for (auto c : g->comms) (void)RC().CommDestroy(c);
  g->be.clear();
  delete g;
}

SVM_API int svmd_cascade_group_world(void* h) { return h ? static_cast<Group*>(h)->world : 0; }

SVM_API svm_cascade_out* svmd_cascade_group_fit(void* h, const void* X, int32_t u8, const int32_t* y, int64_t n,
                                                int64_t d, const svm_cascade_cfg* c) {
  auto* g = static_cast<Group*>(h);
  if (!g || n < 0 || d <= 0 || (n && (!X || !y))) {
    set_error("svmd_cascade_group_fit: bad arguments");
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(g->mu);
  if (g->broken) {
    set_error("svmd_cascade_group_fit: the group's communicators were aborted by an earlier failure; create a new group");
    return nullptr;
  }
  try {
    if (const char* e = getenv("SVM355_CASCADE_PROFILE"); e && atoi(e) >= 3) {
      const auto a = std::chrono::steady_clock::now();
      for (int dv : g->devices) {
        (void)hipSetDevice(dv);
        (void)hipDeviceSynchronize();
      }
      fprintf(stderr, "[svmd_cascade_group_fit] device sync at entry %.3f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count());
    }
    const auto t_setup = std::chrono::steady_clock::now();
    const CascadeConfig cfg = config_from(c);
    const int P = g->world;
    auto token = std::make_shared<AbortToken>();
    const WaitPolicy wp{token, (c && c->comm_timeout_s > 0) ? c->comm_timeout_s : g->timeout_s};
    std::vector<Transport*> tr(static_cast<size_t>(P));
    std::vector<std::unique_ptr<LoopbackTransport>> ltr;
    std::shared_ptr<LoopbackGroup> lg = g->rccl ? nullptr : std::make_shared<LoopbackGroup>(P, wp);
    for (int r = 0; r < P; ++r) {
      if (g->rccl) {
        g->rtr[size_t(r)]->set_policy(wp);
        tr[size_t(r)] = g->rtr[size_t(r)].get();
      } else {
        ltr.push_back(std::make_unique<LoopbackTransport>(lg, r, g->be[size_t(r)].get()));
        tr[size_t(r)] = ltr.back().get();
      }
    }
    const auto t_run = std::chrono::steady_clock::now();
    const size_t row_bytes = u8 ? size_t(d) : size_t(d) * 8;
    std::vector<CascadeOutput> outs(static_cast<size_t>(P));
    std::vector<double> job_in(static_cast<size_t>(P)), job_out(static_cast<size_t>(P));
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    try {
      g->pool->run(
          token,
          [&](int r) {
            const auto tj = std::chrono::steady_clock::now();
            job_in[size_t(r)] = ms(t_run, tj);
            if (hipSetDevice(g->devices[size_t(r)]) != hipSuccess) throw CascadeError("hipSetDevice failed");
            int64_t lo = 0, hi = 0;
            const std::vector<int64_t> ids = partition_ids(n, P, r, &lo, &hi);
            outs[size_t(r)] = run_cascade(*tr[size_t(r)], *g->be[size_t(r)],
                                          static_cast<const char*>(X) + size_t(lo) * row_bytes, u8 != 0, y + lo,
                                          ids.data(), hi - lo, d, n, cfg);
            job_out[size_t(r)] = ms(tj, std::chrono::steady_clock::now());
          },
          [&](int r) {
            (void)hipSetDevice(g->devices[size_t(r)]);
            tr[size_t(r)]->abort();
          });
    } catch (...) {
      if (g->rccl) g->broken = true;  // ncclCommAbort released the communicators
      throw;
    }
    std::vector<const CascadeOutput*> ptrs;
    for (const auto& o : outs) ptrs.push_back(&o);
    (void)hipSetDevice(g->devices[0]);
    const auto t_out = std::chrono::steady_clock::now();
    svm_cascade_out* res = build_cascade_out(ptrs, *g->be[0], P, 0, g->rccl ? "rccl" : "loopback", "hip");
    if (const char* e = getenv("SVM355_CASCADE_PROFILE"); e && atoi(e) >= 2)
      fprintf(stderr,
              "[svmd_cascade_group_fit] setup %.3f ms, ranks %.3f ms (rank 0: woke after %.3f ms, job %.3f ms, "
              "driver %.3f ms), output %.3f ms\n",
              ms(t_setup, t_run), ms(t_run, t_out), job_in[0], job_out[0], outs[0].train_ms,
              ms(t_out, std::chrono::steady_clock::now()));
    return res;
  } catch (const std::exception& e) {
    set_error("cascade: %s", e.what());
    return nullptr;
  }
}

// Distributed decomposition SMO over the group's ranks: every rank's GPU holds all n uint8 rows (host
// X, n x d) and owns a block range of f; one candidate all-gather per outer iteration.  alpha_out
// (host, n doubles) and r come from rank 0 (every rank's alpha is the same replica); stats: SVM_DECOMP_STATS int64
// (decomp.h) from rank 0; rank_ms (world doubles, may be null): each rank's wall time; mm_out (2 d
// doubles, may be null): the column min / max the model's scaling uses.
static int group_decomp(void* h, const void* X, bool u8, const int32_t* y, int64_t n, int64_t d, const svm_params* pp,
                        int32_t q, double* alpha_out, svm_result* r, int64_t* stats, double* rank_ms, double* mm_out) {
  auto* g = static_cast<Group*>(h);
  if (!g || !X || !y || n < 2 || d <= 0) {
    set_error("svmd_cascade_group_decomp: bad arguments");
    return SVM_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(g->mu);
  if (g->broken) {
    set_error("svmd_cascade_group_decomp: the group's communicators were aborted by an earlier failure");
    return SVM_ERR_ARG;
  }
  svm_params p;
  if (pp)
    p = *pp;
  else
    svm_default_params(&p);
  const int P = g->world;
  auto token = std::make_shared<AbortToken>();
  const WaitPolicy wp{token, g->timeout_s};
  std::vector<Transport*> tr(static_cast<size_t>(P));
  std::vector<std::unique_ptr<LoopbackTransport>> ltr;
  std::shared_ptr<LoopbackGroup> lg = g->rccl ? nullptr : std::make_shared<LoopbackGroup>(P, wp);
  for (int rr = 0; rr < P; ++rr) {
    if (g->rccl) {
      g->rtr[size_t(rr)]->set_policy(wp);
      tr[size_t(rr)] = g->rtr[size_t(rr)].get();
    } else {
      ltr.push_back(std::make_unique<LoopbackTransport>(lg, rr, g->be[size_t(rr)].get()));
      tr[size_t(rr)] = ltr.back().get();
    }
  }
  std::vector<double> ms(static_cast<size_t>(P), 0.0);
  const char* serial = getenv("SVM355_CASCADE_SERIAL_SOLVES");
  std::vector<DecompSolo> solo(static_cast<size_t>(serial && atoi(serial) != 0 && !g->rccl && P > 1 ? P : 0));
  for (auto& sr : solo) sr.mu = &g->solo_mu;
  g->solo_report.clear();
  g->host_wait_ms.assign(size_t(P), 0.0);
  try {
    g->pool->run(
        token,
        [&](int rr) {
          if (hipSetDevice(g->devices[size_t(rr)]) != hipSuccess) throw CascadeError("hipSetDevice failed");
          decomp_on_rank(*g->be[size_t(rr)], P > 1 ? tr[size_t(rr)] : nullptr, X, u8, y, n, d, p, q,
                         rr == 0 ? alpha_out : nullptr, rr == 0 ? r : nullptr, rr == 0 ? stats : nullptr,
                         &ms[size_t(rr)], rr == 0 ? mm_out : nullptr, solo.empty() ? nullptr : &solo[size_t(rr)],
                         &g->host_wait_ms[size_t(rr)]);
        },
        [&](int rr) {
          (void)hipSetDevice(g->devices[size_t(rr)]);
          tr[size_t(rr)]->abort();
        });
  } catch (const std::exception& e) {
    if (g->rccl) g->broken = true;
    set_error("decomposition SMO: %s", e.what());
    return SVM_ERR_DEVICE;
  }
  if (rank_ms)
    for (int rr = 0; rr < P; ++rr) rank_ms[rr] = ms[size_t(rr)];
  if (!solo.empty()) {
    // critical path of P GPUs: per outer iteration the slowest rank's selection, then the slowest
    // rank's rest (the ranks meet at the candidate all-gather in between); exchanges excluded
    size_t iters = solo[0].sel_ms.size();
    for (const auto& sr : solo) iters = std::min({iters, sr.sel_ms.size(), sr.rest_ms.size()});
    double sel = 0.0, rest = 0.0;
    for (size_t k = 0; k < iters; ++k) {
      double ms_sel = 0.0, ms_rest = 0.0;
      for (const auto& sr : solo) {
        ms_sel = std::max(ms_sel, sr.sel_ms[k]);
        ms_rest = std::max(ms_rest, sr.rest_ms[k]);
      }
      sel += ms_sel;
      rest += ms_rest;
    }
    g->solo_report = {sel + rest, sel, rest, double(iters)};
    for (const auto& sr : solo) {  // then per rank: its own selection and rest totals
      double a = 0.0, b = 0.0;
      for (double v : sr.sel_ms) a += v;
      for (double v : sr.rest_ms) b += v;
      g->solo_report.push_back(a);
      g->solo_report.push_back(b);
    }
  }
  return SVM_OK;
}

SVM_API int svmd_cascade_group_decomp(void* h, const uint8_t* X, const int32_t* y, int64_t n, int64_t d,
                                      const svm_params* pp, int32_t q, double* alpha_out, svm_result* r,
                                      int64_t* stats, double* rank_ms, double* mm_out) {
  return group_decomp(h, X, true, y, n, d, pp, q, alpha_out, r, stats, rank_ms, mm_out);
}

// The same over FP64 rows (host X, n x d, unscaled): real-valued data train with FP64-MFMA kernel values
// (decomp_fit_rows), pixel values held as doubles with the exact-integer plan.
SVM_API int svmd_cascade_group_decomp_rows(void* h, const double* X, const int32_t* y, int64_t n, int64_t d,
                                           const svm_params* pp, int32_t q, double* alpha_out, svm_result* r,
                                           int64_t* stats, double* rank_ms, double* mm_out) {
  return group_decomp(h, X, false, y, n, d, pp, q, alpha_out, r, stats, rank_ms, mm_out);
}

// The last distributed decomposition fit's host time per rank blocked in the per-batch waits (the one
// wait per outer iteration: RCCL's event poll under the deadline, or hipEventSynchronize); returns P.
SVM_API int64_t svmd_cascade_group_decomp_waits(void* h, double* out, int64_t cap) {
  auto* g = static_cast<Group*>(h);
  if (!g) return 0;
  std::lock_guard<std::mutex> lk(g->mu);
  const int64_t k = std::min<int64_t>(cap, int64_t(g->host_wait_ms.size()));
  for (int64_t i = 0; i < k; ++i) out[i] = g->host_wait_ms[size_t(i)];
  return int64_t(g->host_wait_ms.size());
}

// The last distributed decomposition fit's solo timing on a loopback rehearsal (SVM355_CASCADE_SERIAL_SOLVES=1):
// out = [critical path ms, of it selection ms, of it the rest ms, outer iterations, then per rank: its
// selection ms, its rest ms]; returns the number of values (0: the last fit was not timed solo).
SVM_API int64_t svmd_cascade_group_decomp_solo(void* h, double* out, int64_t cap) {
  auto* g = static_cast<Group*>(h);
  if (!g) return 0;
  std::lock_guard<std::mutex> lk(g->mu);
  const int64_t k = std::min<int64_t>(cap, int64_t(g->solo_report.size()));
  for (int64_t i = 0; i < k; ++i) out[i] = g->solo_report[size_t(i)];
  return int64_t(g->solo_report.size());
}

// One process rank of the distributed decomposition SMO (every rank passes all n rows and labels).
static int rank_decomp(void* h, const void* X, bool u8, const int32_t* y, int64_t n, int64_t d, const svm_params* pp,
                       int32_t q, double* alpha_out, svm_result* r, int64_t* stats, double* ms_out, double* mm_out) {
  auto* pr = static_cast<ProcRank*>(h);
  if (!pr || !X || !y || n < 2 || d <= 0) {
    set_error("svmd_cascade_rank_decomp: bad arguments");
    return SVM_ERR_ARG;
  }
  if (pr->broken) {
    set_error("svmd_cascade_rank_decomp: the communicator was aborted by an earlier failure");
    return SVM_ERR_ARG;
  }
  svm_params p;
  if (pp)
    p = *pp;
  else
    svm_default_params(&p);
  try {
    (void)hipSetDevice(pr->device);
    pr->set_policy(WaitPolicy{nullptr, pr->timeout_s});
    try {
      pr->host_wait_ms = 0.0;
      decomp_on_rank(*pr->be, pr->tr->world() > 1 ? pr->tr.get() : nullptr, X, u8, y, n, d, p, q, alpha_out, r,
                     stats, ms_out, mm_out, nullptr, &pr->host_wait_ms);
    } catch (...) {
      pr->tr->abort();  // the peers' waits fail too
      pr->broken = true;
      throw;
    }
    return SVM_OK;
  } catch (const std::exception& e) {
    set_error("decomposition SMO: %s", e.what());
    return SVM_ERR_DEVICE;
  }
}

SVM_API int svmd_cascade_rank_decomp(void* h, const uint8_t* X, const int32_t* y, int64_t n, int64_t d,
                                     const svm_params* pp, int32_t q, double* alpha_out, svm_result* r,
                                     int64_t* stats, double* ms_out, double* mm_out) {
  return rank_decomp(h, X, true, y, n, d, pp, q, alpha_out, r, stats, ms_out, mm_out);
}

// The same over FP64 rows (svmd_cascade_group_decomp_rows).
SVM_API int svmd_cascade_rank_decomp_rows(void* h, const double* X, const int32_t* y, int64_t n, int64_t d,
                                          const svm_params* pp, int32_t q, double* alpha_out, svm_result* r,
                                          int64_t* stats, double* ms_out, double* mm_out) {
  return rank_decomp(h, X, false, y, n, d, pp, q, alpha_out, r, stats, ms_out, mm_out);
}

// The last svmd_cascade_rank_decomp fit's host time blocked in the per-batch waits (ms).
SVM_API double svmd_cascade_rank_decomp_wait(void* h) {
  auto* pr = static_cast<ProcRank*>(h);
  return pr ? pr->host_wait_ms : 0.0;
}

SVM_API int svmd_nccl_unique_id(uint8_t* out, int64_t cap) {
  if (!out || cap < int64_t(sizeof(ncclUniqueId))) {
    set_error("svmd_nccl_unique_id: need %zu bytes", sizeof(ncclUniqueId));
    return SVM_ERR_ARG;
  }
  try {  // RC() throws when RCCL cannot be loaded: never across the C ABI
    ncclUniqueId id;
    const ncclResult_t rc = RC().GetUniqueId(&id);
    if (rc != ncclSuccess) {
      set_error("ncclGetUniqueId: %s", RC().GetErrorString(rc));
      return SVM_ERR_DEVICE;
    }
    std::memcpy(out, &id, sizeof(id));
    return SVM_OK;
  } catch (const std::exception& e) {
    set_error("svmd_nccl_unique_id: %s", e.what());
    return SVM_ERR_DEVICE;
  }
}

SVM_API int64_t svmd_nccl_unique_id_bytes(void) { return int64_t(sizeof(ncclUniqueId)); }

SVM_API void* svmd_cascade_rank_create(int32_t device, const uint8_t* uid, int32_t world, int32_t rank,
                                       double comm_timeout_s) {
  try {
    if (!uid || world < 1 || rank < 0 || rank >= world) throw CascadeError("bad arguments");
    auto p = std::make_unique<ProcRank>();
    p->device = device;
    p->timeout_s = timeout_or_default(comm_timeout_s);
    if (hipSetDevice(device) != hipSuccess) throw CascadeError("hipSetDevice(" + std::to_string(device) + ") failed");
    p->be = std::make_unique<HipBackend>(device);
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    const ncclResult_t rc = RC().CommInitRank(&p->comm, world, id, rank);
    if (rc != ncclSuccess) throw CascadeError(std::string("ncclCommInitRank: ") + RC().GetErrorString(rc));
    auto rt = std::make_unique<RcclTransport>(p->comm, device, p->be->stream(), WaitPolicy{nullptr, p->timeout_s});
    p->rccl = rt.get();
    p->tr = std::move(rt);
    require_rccl_runtime();
    if (preflight_enabled()) {
      p->set_policy(WaitPolicy{nullptr, kPreflightTimeout});
      try {
        exercise_transport(*p->tr, *p->be, preflight_script(world, kPreflightBytes));
      } catch (const std::exception& e) {
        p->tr->abort();  // the peers' preflight waits fail too
        p->broken = true;
        ProcRank* raw = p.release();
        svmd_cascade_rank_destroy(raw);
        throw CascadeError(std::string("RCCL preflight failed: ") + e.what());
      }
      p->set_policy(WaitPolicy{nullptr, p->timeout_s});
    }
    return p.release();
  } catch (const std::exception& e) {
    set_error("svmd_cascade_rank_create: %s", e.what());
    return nullptr;
  }
}

// A process rank on `device` whose exchanges run through the caller's host collectives (e.g. a gloo
// group under torchrun), device buffers staged through host memory (hostcomm.cpp).  Any number of
// processes may share one GPU: the per-process path of the N-GPU run (the distributed decomposition,
// the cascades) rehearsed on one device.  The callbacks must outlive the rank.  A preflight of the
// driver's op set runs first (collective: every rank creates its rank at the same time).
SVM_API void* svmd_cascade_rank_create_hostcomm(const svm_host_comm* comm, int32_t device, double comm_timeout_s) {
  try {
    if (!host_comm_valid(comm)) throw CascadeError("bad communicator");
    auto p = std::make_unique<ProcRank>();
    p->device = device;
    p->timeout_s = timeout_or_default(comm_timeout_s);
    if (hipSetDevice(device) != hipSuccess) throw CascadeError("hipSetDevice(" + std::to_string(device) + ") failed");
    p->be = std::make_unique<HipBackend>(device);
    p->tr = make_hostcomm_transport(*comm, p->be.get());
    if (preflight_enabled()) {
      try {
        exercise_transport(*p->tr, *p->be, preflight_script(comm->world, kPreflightBytes));
      } catch (const std::exception& e) {
        throw CascadeError(std::string("hostcomm preflight failed: ") + e.what());
      }
    }
    return p.release();
  } catch (const std::exception& e) {
    set_error("svmd_cascade_rank_create_hostcomm: %s", e.what());
    return nullptr;
  }
}

SVM_API void svmd_cascade_rank_destroy(void* h) {
  auto* p = static_cast<ProcRank*>(h);
  if (!p) return;
  (void)hipSetDevice(p->device);
  const bool aborted = p->broken;
  p->tr.reset();
  if (p->comm && !aborted) (void)RC().CommDestroy(p->comm);
  p->be.reset();
  delete p;
}

SVM_API svm_cascade_out* svmd_cascade_rank_fit(void* h, const void* X, int32_t u8, const int32_t* y,
                                               const int64_t* ids, int64_t n_part, int64_t d, int64_t n_total,
                                               const svm_cascade_cfg* c) {
  auto* p = static_cast<ProcRank*>(h);
  if (!p || n_part < 0 || d <= 0 || (n_part && (!X || !y || !ids))) {
    set_error("svmd_cascade_rank_fit: bad arguments");
    return nullptr;
  }
  if (p->broken) {
    set_error("svmd_cascade_rank_fit: the communicator was aborted by an earlier failure");
    return nullptr;
  }
  try {
    (void)hipSetDevice(p->device);
    const CascadeConfig cfg = config_from(c);
    const WaitPolicy wp{nullptr, (c && c->comm_timeout_s > 0) ? c->comm_timeout_s : p->timeout_s};
    p->set_policy(wp);
    CascadeOutput o;
    try {
      o = run_cascade(*p->tr, *p->be, X, u8 != 0, y, ids, n_part, d, n_total, cfg);
    } catch (...) {
      p->tr->abort();  // MPI_Abort equivalent: release the communicator so the peers' waits fail
      p->broken = true;
      throw;
    }
    return build_cascade_out({&o}, *p->be, p->tr->world(), p->tr->rank(), p->tr->name(), "hip");
  } catch (const std::exception& e) {
    set_error("cascade: %s", e.what());
    return nullptr;
  }
}

SVM_API int svmd_cascade_rank_exercise(void* h, const char* script, double timeout_s) {
  auto* p = static_cast<ProcRank*>(h);
  if (!p || p->broken || !script) {
    set_error("svmd_cascade_rank_exercise: no usable communicator");
    return SVM_ERR_ARG;
  }
  try {
    (void)hipSetDevice(p->device);
    p->set_policy(WaitPolicy{nullptr, timeout_s > 0 ? timeout_s : kPreflightTimeout});
    exercise_transport(*p->tr, *p->be, script);
    p->set_policy(WaitPolicy{nullptr, p->timeout_s});
    return SVM_OK;
  } catch (const std::exception& e) {
    p->tr->abort();
    p->broken = true;
    set_error("%s", e.what());
    return SVM_ERR_DEVICE;
  }
}

SVM_API int svmd_cascade_rank_barrier(void* h) {
  auto* p = static_cast<ProcRank*>(h);
  if (!p || p->broken) {
    set_error("svmd_cascade_rank_barrier: no usable communicator");
    return SVM_ERR_ARG;
  }
  try {
    (void)hipSetDevice(p->device);
    p->tr->barrier();
    return SVM_OK;
  } catch (const std::exception& e) {
    set_error("svmd_cascade_rank_barrier: %s", e.what());
    return SVM_ERR_DEVICE;
  }
}

}  // extern "C"

SVMD_TU_WARM(cascade_dev)
