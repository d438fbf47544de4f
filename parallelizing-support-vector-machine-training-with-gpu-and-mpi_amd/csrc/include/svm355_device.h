// svm355 device library C ABI (libsvm355_hip.so, gfx950 / MI355X).
//
// All pointers named *_d are device pointers; every operation is enqueued on the context's
// stream (optionally chained after an external stream, e.g. PyTorch's current stream, through
// svmd_set_stream).  Feature matrices live on the device as row-major n x ld arrays with
// ld = round_up(d, 16) and zero padding (svmd_padded_dim).
//
// Reference parity map (/root/reference/code):
//   svmd_preprocess  <- find_min_max + scale_features kernels  gpu_svm_main3.cu:62-116, 557-598
//   svmd_rbf_gram    <- calc_kernel_matrix (one row at a time) gpu_svm_main3.cu:137-147; here the
//                       whole RBF Gram (or a cross-kernel block) on MFMA f64 tiles
//   svmd_smo         <- SMO_train host loop + WSS/update kernels gpu_svm_main3.cu:152-272, 318-483;
//                       here device-resident: fused f-update+WSS kernel + single-block step kernel,
//                       replayed from a hipGraph with no per-iteration host round trip
//   svmd_decision    <- predict + reduce_sum                   gpu_svm_main3.cu:277-315 (over SVs
//                       only, MFMA cross-kernel + deterministic GEMV)
#pragma once
#include <stdint.h>

#include "svm355.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct svmd_timing {
  double h2d_ms, preprocess_ms, gram_ms, smo_ms, total_ms;
} svmd_timing;

SVM_API int64_t svmd_padded_dim(int64_t d);
SVM_API int svmd_device_count(int32_t* count);

// Plain device memory helpers for native callers that do not link the HIP runtime themselves.
SVM_API void* svmd_alloc(void* ctx, int64_t bytes);
SVM_API void svmd_free(void* ctx, void* ptr);
SVM_API int svmd_memcpy_h2d(void* ctx, void* dst_d, const void* src_h, int64_t bytes);
SVM_API int svmd_memcpy_d2h(void* ctx, void* dst_h, const void* src_d, int64_t bytes);  // synchronous

SVM_API void* svmd_create(int32_t device);
SVM_API void svmd_destroy(void* ctx);
// Free the Gram matrix the library allocated for svmd_train* with K_d == NULL (it is kept in the
// context between calls so repeated fits of the same size do not re-allocate it).
SVM_API int svmd_release_cache(void* ctx);
// Free only the row-cache slab the context keeps after a row-cache fit (see svmd_train_rows).
SVM_API int svmd_release_slab(void* ctx);
// Bytes the context holds for its library-owned Gram and row-cache slab.
SVM_API int svmd_cache_bytes(void* ctx, int64_t* gram, int64_t* slab);
// Size the context-owned Gram for an n-row solve ahead of it (SVM_ERR_OOM if it does not fit).
SVM_API int svmd_reserve_gram(void* ctx, int64_t n);
// Exact-integer training straight from uint8 pixel rows (n x d contiguous, device): *used = 0 and
// nothing done when the rows' statistics do not admit the integer plan (use the FP64-row path).
SVM_API int svmd_train_u8(void* ctx, const uint8_t* Xu_d, int64_t n, int64_t d, const double* mn_h,
                          const double* mx_h, const int32_t* y_d, double* alpha_d, int32_t warm,
                          const svm_params* p, svm_result* r, double* K_d, int64_t ldk, svmd_timing* timing,
                          int32_t* used);
// Working-set decomposition SMO (decomp.hip, opt-in): working sets of up to q <= 1024 points solved
// in one workgroup, f updated by the exact-integer kernel values against the working set; no stored
// Gram.  *used = 0 when the rows are not integer pixels.  stats (optional, 8 int64): outer
// iterations, inner iterations, working-set size, solve microseconds, f-update columns (points
// moved, summed over the outer iterations), inner workgroup size.
SVM_API int svmd_train_decomp_u8(void* ctx, const uint8_t* Xu_d, int64_t n, int64_t d, const double* mn_h,
                                 const double* mx_h, const int32_t* y_d, double* alpha_d, const svm_params* p,
                                 int32_t q, svm_result* r, svmd_timing* timing, int64_t* stats, int32_t* used);
// The same solve from min-max scaled FP64 rows on the device (X_d: n x ld, scaled with the training
// statistics mn_h / mx_h, e.g. by svmd_preprocess): quantised into the same integers as the uint8 path,
// so the model is identical.  *used = 0 when the values admit no exact-integer plan.
SVM_API int svmd_train_decomp_rows(void* ctx, const double* X_d, int64_t n, int64_t ld, int64_t d,
                                   const double* mn_h, const double* mx_h, const int32_t* y_d, double* alpha_d,
                                   const svm_params* p, int32_t q, svm_result* r, svmd_timing* timing,
                                   int64_t* stats, int32_t* used);
SVM_API int svmd_minmax_u8(void* ctx, const uint8_t* Xu_d, int64_t n, int64_t d, double* mn_d, double* mx_d);
SVM_API int svmd_rbf_gram_u8(void* ctx, const uint8_t* Xu_d, int64_t n, int64_t d, const double* mn_h,
                             const double* mx_h, double gamma, double* K_d, int64_t ldk, int32_t* used);
SVM_API int svmd_sv_rows_u8(void* ctx, const uint8_t* Xu_d, int64_t d, const int64_t* idx_d, int64_t k,
                            const double* mn_d, const double* mx_d, double* out_d, int64_t ld, double* sqn_d);
// Self-test of the Gram epilogue's exp: lib_d[i] = device libm exp(x_d[i]), batch_d[i] = the
// batched evaluation the Gram kernel uses (they must agree bit for bit).
SVM_API int svmd_selftest_exp(void* ctx, const double* x_d, int64_t n, double* lib_d, double* batch_d);
// stream = hipStream_t of the caller (may be NULL = legacy default stream).  Work enqueued by the
// context is ordered after everything already on that stream, and the caller's stream waits for
// the context's work before each call returns.
SVM_API int svmd_set_stream(void* ctx, void* stream);
SVM_API int svmd_synchronize(void* ctx);

// Host (n x d, contiguous) -> device (n x ld, zero-padded).  X_d must hold n*ld doubles.
SVM_API int svmd_upload_rows(void* ctx, const double* X_host, int64_t n, int64_t d, double* X_d, int64_t ld);
// Compact uint8 rows (n x d) -> zero-padded FP64 rows on the device (pixel data: 8x less H2D traffic).
SVM_API int svmd_upload_rows_u8(void* ctx, const uint8_t* X_host, int64_t n, int64_t d, double* X_d, int64_t ld);

// Column min/max over n rows (unless use_given != 0, then mn_d/mx_d are inputs), in-place min-max
// scaling with the range < 1e-12 -> 1 rule, and squared row norms sqn_d (length n, may be NULL).
SVM_API int svmd_minmax(void* ctx, const double* X_d, int64_t n, int64_t d, int64_t ld, double* mn_d,
                        double* mx_d);
SVM_API int svmd_preprocess(void* ctx, double* X_d, int64_t n, int64_t d, int64_t ld, double* mn_d,
                            double* mx_d, double* sqn_d, int32_t use_given);
SVM_API int svmd_row_norms(void* ctx, const double* X_d, int64_t n, int64_t d, int64_t ld, double* sqn_d);

// K[i][j] = exp(-gamma * max(0, nA_i + nB_j - 2 A_i.B_j)) for i < m, j < n (row stride ldk).
// sym_diag != 0 forces K[i][i] = 1 (use when A == B).  kdim must be a multiple of 16.
SVM_API int svmd_rbf_gram(void* ctx, const double* A_d, const double* nA_d, int64_t m, int64_t lda,
                          const double* B_d, const double* nB_d, int64_t n, int64_t ldb, int64_t kdim,
                          double gamma, double* K_d, int64_t ldk, int32_t sym_diag);

// SMO on a device kernel matrix.  alpha_d in/out (length n); y_d int32 +-1.
// trace_host (optional): (i_high, i_low) per update, up to trace_cap pairs.
SVM_API int svmd_smo(void* ctx, const double* K_d, int64_t ldk, const int32_t* y_d, int64_t n,
                     double* alpha_d, int32_t warm, const svm_params* p, svm_result* r,
                     int64_t* trace_host, int64_t trace_cap);

// nclass independent cold-start SMO solves on one device kernel matrix (one-vs-rest): Y_d and A_d
// are nclass x n, class-major (row k = class k's +-1 labels / alphas).  The classes run
// concurrently, one XCD-local team of workgroups per XCD pulling classes from a queue; r receives
// nclass results.  *batched (optional) = 1 when the batched kernel ran (else the solves ran one by
// one, e.g. SVM355_SMO_MULTI=0 or a shape it does not cover).
SVM_API int svmd_smo_multi(void* ctx, const double* K_d, int64_t ldk, const int32_t* Y_d, int64_t n, int32_t nclass,
                           double* A_d, const svm_params* p, svm_result* r, int32_t* batched);

// End-to-end training on preprocessed device rows: RBF Gram (allocated internally, or K_d if
// non-NULL with ldk >= n) + SMO.  timing may be NULL.
SVM_API int svmd_train(void* ctx, const double* X_d, const double* sqn_d, int64_t n, int64_t ld,
                       int64_t kdim, const int32_t* y_d, double* alpha_d, int32_t warm,
                       const svm_params* p, svm_result* r, double* K_d, int64_t ldk,
                       svmd_timing* timing);

// As svmd_train, with the Gram path selectable: gram_mode 0 = auto (exact-integer int8-MFMA Gram when
// the scaled rows are integer multiples of 1/(mx_j - mn_j) in [0, 255] — MNIST pixels — else FP64),
// 1 = FP64 only, 2 = integer path required.  mn_h/mx_h: host min/max (d values) the rows were
// scaled with (NULL -> FP64).  *gram_used (optional) = 1 if the integer path ran.
SVM_API int svmd_train_q(void* ctx, const double* X_d, const double* sqn_d, int64_t n, int64_t ld,
                         int64_t kdim, const int32_t* y_d, double* alpha_d, int32_t warm,
                         const svm_params* p, svm_result* r, double* K_d, int64_t ldk,
                         svmd_timing* timing, const double* mn_h, const double* mx_h, int64_t d,
                         int32_t gram_mode, int32_t* gram_used);

// SMO for problems whose Gram does not fit in HBM: kernel rows are computed on demand into a 2-way
// set-associative LRU row cache of cache_bytes (<= 0: 16384 rows, at most 60% of the free HBM), filled by a grid-wide
// kernel inside the replayed iteration graph (rowcache.hip).  With integer-valued rows the values
// are bit-identical to the exact-integer Gram (same trajectory as svmd_train_q); otherwise FP64
// rows (sqn_d required).  d = feature count (FP64 rows use the first d columns).
SVM_API int svmd_train_rows(void* ctx, const double* X_d, const double* sqn_d, int64_t n, int64_t ld,
                            int64_t d, const int32_t* y_d, double* alpha_d, int32_t warm,
                            const svm_params* p, svm_result* r, const double* mn_h, const double* mx_h,
                            int32_t gram_mode, int64_t cache_bytes, int32_t* gram_used,
                            int64_t* trace_host, int64_t trace_cap);

// Symmetric RBF Gram of n preprocessed rows with the same path selection as svmd_train_q.
SVM_API int svmd_rbf_gram_q(void* ctx, const double* X_d, const double* sqn_d, int64_t n, int64_t ld,
                            int64_t kdim, const double* mn_h, const double* mx_h, int64_t d,
                            double gamma, double* K_d, int64_t ldk, int32_t gram_mode,
                            int32_t* gram_used);

// out_d[i] = sum_k coef_d[k] * K(Xq_i, Xs_k) - b, coef = alpha*y of the SVs.
SVM_API int svmd_decision(void* ctx, const double* Xs_d, const double* ns_d, const double* coef_d,
                          int64_t nsv, int64_t lds, const double* Xq_d, const double* nq_d, int64_t m,
                          int64_t ldq, int64_t kdim, double gamma, double b, double* out_d);

// out_d[i] = sum_{k < nz} coef_d[k] * K(X_i, X_k) for the k (scaled) rows X_d whose first nz rows are
// the terms, on the exact-integer path (the Gram's kernel values; mn_h / mx_h: host column
// statistics the rows were scaled with).  *used = 0 (nothing written) when the rows are not
// integer-valued pixels: the caller then takes svmd_decision.
SVM_API int svmd_decision_int(void* ctx, const double* X_d, int64_t k, int64_t ldx, int64_t d, const double* mn_h,
                              const double* mx_h, const double* coef_d, int64_t nz, double gamma, double* out_d,
                              int32_t* used);

// *correct = #{i : sign(dec_d[i]) == y_d[i]} on the device (prediction accuracy numerator);
// zero_positive = 1 maps s >= 0 to +1 (cascade programs), 0 maps s > 0 to +1 (serial / GPU programs).
SVM_API int svmd_count_correct(void* ctx, const double* dec_d, const int32_t* y_d, int64_t m,
                               int32_t zero_positive, int64_t* correct);

// dst[k] = src[idx[k]] rows (device gather), for SV compaction and cascade training-set assembly.
SVM_API int svmd_gather_rows(void* ctx, const double* src_d, int64_t ld, const int64_t* idx_d,
                             int64_t k, double* dst_d);

// ---- Cascade SVM on MI355X GPUs (csrc/hip/cascade_dev.hip; round logic in csrc/cascade).
// Thread-rank group of this process: world ranks on GPUs 0..world-1 with one RCCL communicator each
// (ncclCommInitAll over xGMI, transport "rccl"), or world ranks sharing the visible GPUs with
// host-staged exchanges ("loopback", a rehearsal of any P on one GPU); "auto" = rccl when world
// GPUs are visible.  fit partitions X (n x d, float64 or uint8 pixels when u8) into contiguous
// ceil(n / world) chunks with global ids; the group keeps its contexts / buffers between fits.
SVM_API void* svmd_cascade_group_create(int32_t world, const char* transport, double comm_timeout_s);
SVM_API int svmd_cascade_group_world(void* group);
SVM_API svm_cascade_out* svmd_cascade_group_fit(void* group, const void* X, int32_t u8, const int32_t* y, int64_t n,
                                                int64_t d, const svm_cascade_cfg* cfg);
SVM_API void svmd_cascade_group_destroy(void* group);
// One rank per process (e.g. torchrun): rank 0 makes the id, the launcher distributes it.
SVM_API int64_t svmd_nccl_unique_id_bytes(void);
SVM_API int svmd_nccl_unique_id(uint8_t* out, int64_t cap);
SVM_API void* svmd_cascade_rank_create(int32_t device, const uint8_t* uid, int32_t world, int32_t rank,
                                       double comm_timeout_s);
// The same rank over caller-supplied host collectives (svm_host_comm: a gloo group under torchrun), its
// device buffers staged through host memory; several processes may share one GPU (the per-process
// launch rehearsed on one device).  Every rank_* entry point below takes either kind of rank.
// The last svmd_cascade_group_decomp fit's solo timing on a loopback rehearsal with
// SVM355_CASCADE_SERIAL_SOLVES=1 (each rank's device work timed alone): [critical path ms, selection ms,
// rest ms, outer iterations, then per rank: selection ms, rest ms]; returns the count (0: not timed).
SVM_API int64_t svmd_cascade_group_decomp_solo(void* group, double* out, int64_t cap);
// The last svmd_cascade_group_decomp fit's per-rank host time blocked in the per-batch waits (ms);
// returns the number of ranks.
SVM_API int64_t svmd_cascade_group_decomp_waits(void* group, double* out, int64_t cap);
// The same for this process's rank (svmd_cascade_rank_decomp).
SVM_API double svmd_cascade_rank_decomp_wait(void* rank);
SVM_API void* svmd_cascade_rank_create_hostcomm(const svm_host_comm* comm, int32_t device, double comm_timeout_s);
SVM_API svm_cascade_out* svmd_cascade_rank_fit(void* rank, const void* X, int32_t u8, const int32_t* y,
                                               const int64_t* ids, int64_t n_part, int64_t d, int64_t n_total,
                                               const svm_cascade_cfg* cfg);
SVM_API int svmd_cascade_rank_barrier(void* rank);
// RCCL preflight / transport exerciser (csrc/cascade/exercise.cpp script syntax): run `script` with
// checked payloads on every rank of a group (rccl or loopback), or on this process's rank (every
// rank of the communicator calls it collectively).  Group and rank creation already run the
// driver's op set (svm_preflight_script) on RCCL communicators (SVM355_RCCL_PREFLIGHT=0 skips it).
// A failure aborts the communicators (the group / rank is then unusable).
SVM_API int svmd_cascade_group_exercise(void* group, const char* script, double timeout_s);
// Distributed working-set decomposition SMO (decomp.hip) over a group's ranks or one process rank:
// every rank's GPU holds all n uint8 rows (host X, n x d) and labels, owns a block range of f, and
// all-gathers its candidate records once per outer iteration; the working set, inner solve and alpha
// are replicated.  With 1, 2, 4 or 8 ranks the trajectory equals svmd_train_decomp_u8's.  alpha_out
// (n), r, stats (8 int64, see svmd_train_decomp_u8) and mm_out (2 d: column min / max) may be null.
SVM_API int svmd_cascade_group_decomp(void* group, const uint8_t* X, const int32_t* y, int64_t n, int64_t d,
                                      const svm_params* p, int32_t q, double* alpha_out, svm_result* r,
                                      int64_t* stats, double* rank_ms, double* mm_out);
SVM_API int svmd_cascade_rank_decomp(void* rank, const uint8_t* X, const int32_t* y, int64_t n, int64_t d,
                                     const svm_params* p, int32_t q, double* alpha_out, svm_result* r,
                                     int64_t* stats, double* ms_out, double* mm_out);
SVM_API int svmd_cascade_rank_exercise(void* rank, const char* script, double timeout_s);
SVM_API int svmd_cascade_group_broken(void* group);  // 1 once a failure aborted its communicators
// RCCL the library was compiled against (NCCL_VERSION_CODE) and the one it runs on (ncclGetVersion),
// with the path of the loaded librccl (in a PyTorch process: usually torch's bundled copy).
SVM_API int svmd_rccl_info(int32_t* header_code, int32_t* runtime_code, char* path, int64_t cap);
SVM_API void svmd_cascade_rank_destroy(void* rank);

// ---- Distributed SMO (csrc/hip/dsmo.hip): ONE first-order SMO whose training points are split
// over `world` teams -- one per GPU (rehearsal = 0: GPUs 0..world-1 of this process, peer access
// between them) or all on GPU 0 (rehearsal != 0, one launch) -- each holding its slab K(:, own) of
// the exact-integer Gram and exchanging the per-iteration candidates over xGMI.  The trajectory
// (every pair, alpha and b) is the single-GPU resident solve's.  X: n x d uint8 pixel rows (host).
// alpha_out: n doubles (host); timing_out (optional, 4 doubles): slowest GPU's upload+min/max,
// quantise+slabs, solve and total ms; trace (optional, host): (i_high, i_low) per update;
// shape_out (optional, 4 ints): threads per workgroup, points per thread, workgroups per team,
// records per sweep lane; mn_out / mx_out (optional, d doubles each): the column statistics.
SVM_API void* svmd_dsmo_create(int32_t world, int32_t rehearsal, double timeout_s);
SVM_API void svmd_dsmo_destroy(void* group);
SVM_API int svmd_dsmo_world(void* group);
// Team plan for n points over P teams (ncu CUs per GPU; one_launch != 0: every team co-resident on
// one GPU): out[6] = {threads per workgroup, points per thread, workgroups per team, records per
// sweep lane, points per workgroup, points per team}.  Host only (no device needed).
SVM_API int svmd_dsmo_plan(int64_t n, int32_t P, int32_t ncu, int32_t one_launch, int64_t* out);
SVM_API int svmd_dsmo_fit(void* group, const void* X, int32_t u8, const int32_t* y, int64_t n, int64_t d,
                          const svm_params* p, double* alpha_out, svm_result* r, double* timing_out, int64_t* trace,
                          int64_t trace_cap, int32_t* shape_out, double* mn_out, double* mx_out);
// One team per process (e.g. torchrun): create on this rank's GPU, export the receive array
// (svmd_dsmo_rank_handle, svmd_dsmo_handle_bytes() bytes), all-gather the handles through the
// launcher, connect (opens the peers' arrays over IPC).  A fit = rank_prepare (rows, slab) on every
// rank, a launcher barrier, then rank_solve on every rank (the launch; this rank's alpha slice,
// range_out = its [col0, ncols)).
SVM_API void* svmd_dsmo_rank_create(int32_t device, int32_t world, int32_t rank, double timeout_s);
SVM_API int64_t svmd_dsmo_handle_bytes(void);
SVM_API int svmd_dsmo_rank_handle(void* rank, uint8_t* out, int64_t cap);
SVM_API int svmd_dsmo_rank_connect(void* rank, const uint8_t* handles);
SVM_API int svmd_dsmo_rank_prepare(void* rank, const void* X, int32_t u8, const int32_t* y, int64_t n, int64_t d,
                                   const svm_params* p);
SVM_API int svmd_dsmo_rank_solve(void* rank, double* alpha_out, svm_result* r, double* timing_out, int32_t* shape_out,
                                 double* mn_out, double* mx_out, int64_t* range_out);

// roctx ranges (rocprofv3 --marker-trace); the library already brackets preprocess / gram / smo /
// decision, these let callers mark their own phases (e.g. cascade rounds and exchanges).
SVM_API void svmd_trace_push(const char* name);
SVM_API void svmd_trace_pop(void);

#ifdef __cplusplus
}
#endif
