// Device context: stream, cross-stream ordering and a grow-only workspace.
#pragma once
#include <vector>

#include "hip_util.h"

namespace svm355 {

// The calling thread's current device for the scope, restored on exit: entry points that only free or
// query a context (possibly another GPU's) must not move the caller's (PyTorch's) current device.
struct ScopedDevice {
  int prev = -1;
  explicit ScopedDevice(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~ScopedDevice() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  ScopedDevice(const ScopedDevice&) = delete;
  ScopedDevice& operator=(const ScopedDevice&) = delete;
};

struct DeviceCtx {
  int device = 0;
  hipStream_t stream = nullptr;  // private non-blocking stream (graph-capturable)
  hipStream_t ext = nullptr;     // caller's stream (PyTorch current stream), may be null
  bool has_ext = false;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  hipEvent_t ev_ctl[2] = {nullptr, nullptr};  // decomposition solver: its control readbacks (decomp.hip)
  void* ws = nullptr;
  size_t ws_bytes = 0;
  void* pinned = nullptr;
  size_t pinned_bytes = 0;
  // Library-owned Gram (svmd_train* with K_d == NULL): kept between calls so a repeated fit of the
  // same size neither re-allocates nor frees 10s of GB inside the timed region; freed by
  // svmd_release_cache / svmd_destroy or when a larger one is needed.
  double* gram = nullptr;
  size_t gram_bytes = 0;
  // Row-cache slab (rowcache.hip), kept like the Gram: a large-n fit does not map and unmap tens of
  // GB per call, and the default cache size does not depend on what the last free left unmapped.
  double* rc_cache = nullptr;
  size_t rc_cache_bytes = 0;
  double ccache_frac = -1.0;  // decomposition column cache cap as a fraction of the HBM (< 0: the default)
  unsigned long long* count_d = nullptr;  // device counter for count_sv
  // Cached SMO iteration graph (smo.hip) and the argument key it was captured for.
  hipGraphExec_t smo_exec = nullptr;
  hipGraph_t smo_graph = nullptr;
  std::vector<uint64_t> smo_key;

  void release_graph() {
    if (smo_exec) (void)hipGraphExecDestroy(smo_exec);
    if (smo_graph) (void)hipGraphDestroy(smo_graph);
    smo_exec = nullptr;
    smo_graph = nullptr;
    smo_key.clear();
  }

  // Make the private stream wait for work already enqueued on the caller's stream.
  int begin() {
    SVMD_CHECK(hipSetDevice(device));
    if (has_ext) {
      SVMD_CHECK(hipEventRecord(ev_in, ext));
      SVMD_CHECK(hipStreamWaitEvent(stream, ev_in, 0));
    }
    return SVM_OK;
  }
  // Make the caller's stream wait for the private stream.
  int end() {
    if (has_ext) {
      SVMD_CHECK(hipEventRecord(ev_out, stream));
      SVMD_CHECK(hipStreamWaitEvent(ext, ev_out, 0));
    }
    return SVM_OK;
  }
  int ensure_ws(size_t bytes) {
    if (bytes <= ws_bytes) return SVM_OK;
    if (ws) {
      SVMD_CHECK(hipStreamSynchronize(stream));
      SVMD_CHECK(hipFree(ws));
      ws = nullptr;
      ws_bytes = 0;
    }
    const size_t sz = (bytes + 0xFFFFF) & ~size_t(0xFFFFF);
    SVMD_CHECK(hipMalloc(&ws, sz));
    ws_bytes = sz;
    return SVM_OK;
  }
  double* ensure_rc_cache(size_t bytes) {  // nullptr when the allocation fails
    if (bytes <= rc_cache_bytes) return rc_cache;
    if (rc_cache) {
      if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
      (void)hipFree(rc_cache);
      rc_cache = nullptr;
      rc_cache_bytes = 0;
    }
    if (hipMalloc(&rc_cache, bytes) != hipSuccess) {
      rc_cache = nullptr;
      return nullptr;
    }
    rc_cache_bytes = bytes;
    return rc_cache;
  }
  int ensure_pinned(size_t bytes) {
    if (bytes <= pinned_bytes) return SVM_OK;
    if (pinned) {
      SVMD_CHECK(hipStreamSynchronize(stream));
      SVMD_CHECK(hipHostFree(pinned));
      pinned = nullptr;
      pinned_bytes = 0;
    }
    const size_t sz = (bytes + 0xFFFF) & ~size_t(0xFFFF);
    SVMD_CHECK(hipHostMalloc(&pinned, sz, hipHostMallocDefault));
    pinned_bytes = sz;
    return SVM_OK;
  }
};

#define SVMD_CTX(h)                                              \
  auto* ctx = static_cast<svm355::DeviceCtx*>(h);                 \
  if (!ctx) {                                                    \
    svm355::set_error("null device context");                    \
    return SVM_ERR_ARG;                                          \
  }

// Load every translation unit's code object on s (hip_util.h SVMD_TU_WARM): svmd_create.
int tu_warm_all(hipStream_t s);

// Kernel launchers implemented in the .hip translation units (all enqueue on `s`).
int launch_widen_u8(hipStream_t s, const uint8_t* src, int64_t n, int64_t d, int64_t ld, double* dst);
int launch_minmax(hipStream_t s, const double* X, int64_t n, int64_t d, int64_t ld, double* mn,
                  double* mx, double* scratch, size_t scratch_doubles);
int launch_scale_norms(hipStream_t s, double* X, int64_t n, int64_t d, int64_t ld, const double* mn,
                       const double* mx, double* sqn);
int launch_gather_rows(hipStream_t s, const double* src, int64_t ld, const int64_t* idx, int64_t k,
                       double* dst);
int launch_rbf_gram(hipStream_t s, const double* A, const double* nA, int64_t m, int64_t lda,
                    const double* B, const double* nB, int64_t n, int64_t ldb, int64_t kdim,
                    double gamma, double* K, int64_t ldk, bool sym_diag);
int launch_gemv_rows(hipStream_t s, const double* K, int64_t ldk, int64_t m, int64_t n,
                     const double* coef, double b, double* out);
// K(A rows, B rows) on FP64 MFMA with device-side controls (decomposition solver, FP64 rows): gate !=
// 0 -> no-op; B rows bounded by *ncount (<= ncap; whole workgroups beyond exit); sym_diag: K_ii = 1 by
// position; colid: B row j is training row colid[j], A row i is row_off + i, and that pair's K = 1.
int launch_rbf_block_dev(hipStream_t s, const double* A, const double* nA, int64_t m, int64_t lda, const double* B,
                         const double* nB, int64_t ncap, int64_t ldb, int64_t kdim, double gamma, double* K, int64_t ldk,
                         bool sym_diag, const int32_t* gate, const int32_t* ncount, const int32_t* colid,
                         int64_t row_off);
// Exact-integer Gram path (igram.hip).
struct QuantPlan {
  bool ok = false;
  double w0 = 0.0;            // weight 1/r^2 of the main (exact-integer) column group
  int kq = 0;                 // int8 columns (multiple of 64)
  int main0 = 0;              // first column of the main group (extra groups before it, multiple of 32)
  int n_groups = 0;
  std::vector<int32_t> perm;  // permuted column order (-1 = zero pad)
  std::vector<double> rmul;   // r_j per permuted column (scaled value * r_j = integer)
  std::vector<double> off;    // centring offset floor(r_j / 2)
  std::vector<double> wx;     // 1/r_j^2 for extra-group columns (0 for main / pad)
  std::vector<double> step_w; // per 32-column k-step below main0: group weight at its last step, else 0
};
bool plan_quant(const double* mn, const double* mx, int64_t d, QuantPlan* P);
size_t igram_workspace(int64_t n, const QuantPlan& P);
size_t quantize_aux_bytes(const QuantPlan& P);
int quantize_rows(hipStream_t s, const double* X, int64_t n, int64_t ld, const QuantPlan& P, void* aux, int8_t* Q,
                  int32_t* N0, double* WN, bool* ok);
// copy_stw = false: the step weights are already in stw (no host-to-device copy on the stream).
int launch_igram_sym(hipStream_t s, const int8_t* Q, const int32_t* N0, const double* WN, double* stw, int64_t n,
                     const QuantPlan& P, double gamma, double* K, int64_t ldk, bool copy_stw = true, const int32_t* gate = nullptr);
int launch_igram_slab(hipStream_t s, const int8_t* Q, const int32_t* N0, const double* WN, const double* stw,
                      int64_t n, int64_t col0, int64_t ncols, const QuantPlan& P, double gamma, double* K,
                      int64_t ldk);
int launch_igram_gemv(hipStream_t s, const int8_t* Q, const int32_t* N0, const double* WN, const double* stw,
                      int64_t n, int64_t row_off, const int8_t* Qc, const int32_t* N0c, const double* WNc,
                      const int32_t* cols, const double* coef, const int32_t* mcount, int64_t m, const QuantPlan& P,
                      double gamma, double* part, int64_t ldp, const int32_t* diag = nullptr);
// K(W, W) through the narrow column store; *launched = false (SVM_OK) when its shape limits do not apply.
int launch_igram_ww(hipStream_t s, const int8_t* Qw, const int32_t* N0w, const double* WNw, const double* stw,
                    int64_t n, const int32_t* ids, const int32_t* count, const QuantPlan& P, double gamma, double* K,
                    int64_t ldk, const int32_t* gate, bool* launched);
int launch_igram_colstore(hipStream_t s, const int8_t* Q, const int32_t* N0, const double* WN, const double* stw,
                          int64_t n, int64_t row_off, const int8_t* Qc, const int32_t* N0c, const double* WNc,
                          const int32_t* ids, const int32_t* slots, const int32_t* count, int64_t m,
                          const QuantPlan& P, double gamma, double* cache, int64_t ldc, const int32_t* gate,
                          bool tiled = true, const int32_t* diag = nullptr);
int run_igram_u8(hipStream_t s, const uint8_t* Xu, int64_t n, int64_t d, const double* mn_h, const double* mx_h,
                 const QuantPlan& P, double gamma, double* K, int64_t ldk, void* ws, bool* used);
size_t igram_u8_workspace(int64_t n, const QuantPlan& P);
size_t quantize_u8_aux_bytes(const QuantPlan& P);
int quantize_u8_rows(hipStream_t s, const uint8_t* Xu, int64_t n, int64_t d, const double* mn_h, const double* mx_h,
                     const QuantPlan& P, void* aux, int8_t* Q, int32_t* N0, double* WN, bool* ok);
int launch_minmax_u8(hipStream_t s, const uint8_t* X, int64_t n, int64_t d, double* mn, double* mx, double* scratch,
                     size_t scratch_doubles);
int launch_sv_rows_u8(hipStream_t s, const uint8_t* X, int64_t d, const int64_t* idx, int64_t k, const double* mn,
                      const double* mx, double* out, int64_t ld, double* sqn);
int run_igram(hipStream_t s, const double* X, int64_t n, int64_t ld, const QuantPlan& P, double gamma, double* K,
              int64_t ldk, void* ws, bool* used);
int run_igram_block(hipStream_t s, const double* X, int64_t n, int64_t ld, int64_t ncols, const QuantPlan& P,
                    double gamma, double* K, int64_t ldk, void* ws, bool* used);
int run_smo_rowcache(DeviceCtx* ctx, const double* X_d, const double* sqn_d, int64_t n, int64_t ld, int64_t d,
                     const QuantPlan& P, const int32_t* y, double* alpha, int32_t warm, const svm_params& p,
                     svm_result* r, size_t cache_bytes, int64_t* trace, int64_t trace_cap, int32_t* used_int);
int run_smo(DeviceCtx* ctx, const double* K, int64_t ldk, const int32_t* y, int64_t n, double* alpha,
            int32_t warm, const svm_params& p, svm_result* r, int64_t* trace, int64_t trace_cap);
// Persistent row-cache SMO (smo.hip): f / alpha initialised by the caller; kRcNotApplicable when no
// persistent shape covers n (SVM355_RC_SMO=graph forces that answer).
struct QRows;
constexpr int kRcNotApplicable = -100;
int run_smo_rc_persistent(DeviceCtx* ctx, const QRows& q, bool int_rows, double* cache, int64_t ldc, int64_t nslots,
                          const int32_t* y, double* alpha, double* f, int64_t n, const svm_params& p, svm_result* r,
                          int64_t* trace, int64_t trace_cap);
// nclass cold-start solves on one Gram (Y, A: nclass x n, class-major): XCD teams (smo.hip).
// exp self-test (igram.hip): device libm exp and the Gram epilogue's batched exp of x[0..n).
int exp_selftest(hipStream_t s, const double* x, int64_t n, double* out_lib, double* out_batch);
// Number of alpha[i] > tol for i < n (device reduction; one 8-byte read-back per row of alphas).
int count_sv(DeviceCtx* ctx, const double* alpha, int64_t n, int64_t rows, double tol, int64_t* out);
int count_correct(DeviceCtx* ctx, const double* dec, const int32_t* y, int64_t m, bool zero_positive,
                  int64_t* out);
int run_smo_multi(DeviceCtx* ctx, const double* K, int64_t ldk, const int32_t* Y, int64_t n, int nclass, double* A,
                  const svm_params& p, svm_result* r, int32_t* batched);

}  // namespace svm355
