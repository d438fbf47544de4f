// svm355 — C ABI of the native runtime (CPU core + HIP/gfx950 device library).
//
// Everything the Python package and the native CLIs call goes through this header.
// The CPU core (libsvm355_core.so) implements the reference semantics exactly and
// doubles as the correctness oracle; the device library (libsvm355_hip.so) implements
// the same contract on MI355X with hand-written CDNA4 kernels.
//
// Reference parity map (files under /root/reference/code):
//   svm_csv_load        <- read_CSV                 main3.cpp:13-54, gpu_svm_main4.cu:16-59 (row limit)
//   svm_minmax/scale    <- find_min_max/scale_features main3.cpp:57-89
//   svm_rbf             <- kernel                   main3.cpp:92-104 (gamma made a parameter)
//   svm_smo_train       <- SMO_train                main3.cpp:162-294, warm start mpi_svm_main3.cpp:155-290
//   svm_decision        <- predict loop             main3.cpp:391-402
//   svm_model_save      <- commented model dump     mpi_svm_main3.cpp:754-770
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SVM_API __attribute__((visibility("default")))

enum svm_status {
  SVM_OK = 0,
  SVM_ERR_IO = 1,
  SVM_ERR_ARG = 2,
  SVM_ERR_EMPTY = 3,
  SVM_ERR_DEVICE = 4,
  SVM_ERR_INTERNAL = 5,
  SVM_ERR_OOM = 6,
};

// Why an SMO solve ended. Codes match the reference's stderr messages.
enum svm_stop {
  SVM_STOP_RUNNING = 0,
  SVM_STOP_CONVERGED = 1,     // b_low <= b_high + 2*tau
  SVM_STOP_NO_CANDIDATE = 2,  // "i_high or i_low not found; iteration stops"
  SVM_STOP_INFEASIBLE = 3,    // "warning: infeasible U and V; iteration stops"
  SVM_STOP_NONPOS_ETA = 4,    // "warning: non positive eta; iteration stops"
  SVM_STOP_MAX_ITER = 5,      // "Too many iterations; stopping"
};

typedef struct svm_params {
  double C;          // box constraint, reference default 10
  double gamma;      // RBF width, reference default 0.00125
  double tau;        // stop when b_low <= b_high + 2*tau, default 1e-5
  double eps;        // set-membership / eta floor, default 1e-12
  double sv_tol;     // alpha > sv_tol is a support vector, default 1e-8
  int64_t max_iter;  // default 100000 (num_iter starts at 1)
  int32_t n_threads; // CPU worker threads (1 = the serial reference baseline)
  int32_t verbose;
  int32_t wss;       // working-set selection: 0 / 1 = first order (reference), 2 = second-order j
  int32_t shrink;    // decomposition solver shrinking: 0 = default (off), -1 = off, k > 0 = every k outer
                     // iterations (decomp_shrink.h)
} svm_params;

typedef struct svm_result {
  int64_t iterations;  // the reference's printed num_iter (updates + 1)
  double b;            // (b_high + b_low) / 2
  double b_high;
  double b_low;
  int32_t stop_reason; // enum svm_stop
  int32_t reserved;
  int64_t n_sv;        // alpha > sv_tol
  double seconds;      // solver wall time
} svm_result;

SVM_API const char* svm_last_error(void);
SVM_API void svm_default_params(svm_params* p);
SVM_API const char* svm_stop_message(int32_t reason);

// ---------------------------------------------------------------- data I/O (L0)
// Loads a CSV with a header row; the last column is the integer label.
// limit < 0 reads every line; otherwise at most `limit` data lines are consumed
// (skipped short lines count toward the limit, as gpu_svm_main4.cu:34-38).
// y = +1 where label == positive_label, else -1 (main3.cpp:49-52 with positive_label=1).
SVM_API void* svm_csv_load(const char* path, int64_t limit, int32_t positive_label, int32_t n_threads);
SVM_API int svm_dataset_dims(void* h, int64_t* n, int64_t* d);
SVM_API int svm_dataset_copy(void* h, double* X, int32_t* y, int32_t* raw_labels);
SVM_API void svm_dataset_free(void* h);
SVM_API int svm_csv_write(const char* path, const double* X, const int32_t* labels, int64_t n, int64_t d);

// Deterministic MNIST-shaped generator: 28x28 (d=784) integer pixels 0..255, labels 0..9.
// Writes global samples [offset, offset + n); sample i depends only on (seed, i).
SVM_API int svm_synth_mnist(uint64_t seed, int64_t offset, int64_t n, double* X, int32_t* labels,
                            int32_t n_threads);

// ---------------------------------------------------------------- preprocessing (L1)
SVM_API int svm_minmax(const double* X, int64_t n, int64_t d, double* mn, double* mx);
SVM_API int svm_scale(double* X, int64_t n, int64_t d, const double* mn, const double* mx);

// ---------------------------------------------------------------- kernel (L2)
SVM_API double svm_rbf(const double* a, const double* b, int64_t d, double gamma);
SVM_API int svm_rbf_matrix(const double* A, int64_t m, const double* B, int64_t n, int64_t d,
                           double gamma, double* K, int32_t n_threads);

// ---------------------------------------------------------------- SMO (L3)
// alpha: in/out length n. warm=0: alpha reset to 0 and f = -y (main3.cpp:165-172).
// warm=1: f_i = sum_{alpha_j != 0} alpha_j y_j K_ij - y_i (mpi_svm_main3.cpp:169-186).
// trace (optional, may be NULL): receives (i_high, i_low) for each update, up to trace_cap pairs.
SVM_API int svm_smo_train(const double* X, const int32_t* y, int64_t n, int64_t d, double* alpha,
                          int32_t warm, const svm_params* p, svm_result* r, int64_t* trace,
                          int64_t trace_cap);
// Same solver on a precomputed kernel matrix K (n x n, row stride ldk).
SVM_API int svm_smo_train_gram(const double* K, int64_t ldk, const int32_t* y, int64_t n,
                               double* alpha, int32_t warm, const svm_params* p, svm_result* r,
                               int64_t* trace, int64_t trace_cap);

// ---------------------------------------------------------------- working-set decomposition (L3)
// Per-outer-iteration record of a working-set decomposition solve: the device solver's test trace
// (svmd_train_decomp with a trace) and its CPU oracle's (svm_decomp_train_gram).  Caller-allocated
// arrays for `cap` outer iterations; the stopping build is not recorded.
#define SVM_DECOMP_MAX_WS 1024
// int64 entries of a decomposition solve's stats array: outer / inner iterations, working-set capacity,
// solve us, moved columns, inner threads, kernel-value path, warm columns, unshrinks, shrink passes,
// the least active rows seen, repacks, Newton steps (decomp_shrink.h / decomp_newton.h), 3 reserved
#define SVM_DECOMP_STATS 16
typedef struct svm_decomp_trace {
  int64_t cap;     // capacity in outer iterations
  int64_t count;   // out: outer iterations recorded
  int64_t n;       // length of the alpha / f snapshots (0 = none)
  int32_t* m;      // cap: working-set size
  int32_t* W;      // cap x SVM_DECOMP_MAX_WS: the working set, ascending ids
  int32_t* moved;  // cap: points whose alpha changed in the inner solve
  int32_t* cols;   // cap x SVM_DECOMP_MAX_WS: their ids, ascending
  double* coef;    // cap x SVM_DECOMP_MAX_WS: (alpha_new - alpha_old) y
  int64_t* inner;  // cap: inner iterations (pair updates)
  double* bounds;  // cap x 2: b_high, b_low of the build
  double* alpha;   // cap x n or NULL: alpha after the outer iteration
  double* f;       // cap x n or NULL: f after the outer iteration's update
} svm_decomp_trace;

// CPU oracle of the device decomposition solver (csrc/hip/decomp.hip) on a precomputed kernel matrix
// K (n x n, row stride ldk; the device's own kernel values for a bit-for-bit comparison): the same
// block selection, working-set build and stop test, the inner solve's arithmetic and tie rules, and
// the f update in the device GEMV's summation order.  q: working-set size (<= 1024); tau_frac: inner
// stop fraction (device default 0.1); inner_wss: 3 = second-order second index plus a second pair per
// iteration (device default), 4 = the same with the second pair's j by the second-order gain of
// row i2 (SVM355_DECOMP_WSS=4), 2 = second order alone, 1 = first order.  warm = 1: alpha holds the start and f = K (alpha y) - y over its nonzero entries in
// chunks of 1024 columns (the device's warm start).  stats (8 int64, may be NULL) as the device's:
// outer, inner iterations, working-set capacity, microseconds, moved columns, 0, 0, warm-start columns.
SVM_API int svm_decomp_train_gram(const double* K, int64_t ldk, const int32_t* y, int64_t n, double* alpha,
                                  int32_t warm, const svm_params* p, int32_t q, double tau_frac, int32_t inner_wss,
                                  svm_result* r, int64_t* stats, svm_decomp_trace* trace);

// The device f-update GEMV's arithmetic alone: f[i] += sum_{k < cnt} coef[k] K(i, cols[k]) for the n
// rows of K, in the device's summation order (bit-for-bit tests of the GEMV kernel).
SVM_API int svm_decomp_gemv_ref(const double* K, int64_t ldk, int64_t n, const int32_t* cols, const double* coef,
                                int64_t cnt, double* f);

// ---------------------------------------------------------------- evaluation (L4)
// out[i] = sum_k alphas[k]*ys[k]*K(Xq_i, Xs_k) - b, summed in SV order from -b (main3.cpp:391-402).
SVM_API int svm_decision(const double* Xs, const int32_t* ys, const double* alphas, int64_t nsv,
                         const double* Xq, int64_t m, int64_t d, double gamma, double b,
                         double* out, int32_t n_threads);
// Indices with alpha > tol, ascending; returns the count (out may be NULL to count only).
SVM_API int64_t svm_sv_indices(const double* alpha, int64_t n, double tol, int64_t* out);

// ---------------------------------------------------------------- model files (C31)
// Writes final_sv_ids.txt, final_sv_labels.txt, final_sv_alphas.txt, final_b.txt into dir.
SVM_API int svm_model_save(const char* dir, const int64_t* ids, const int32_t* labels,
                           const double* alphas, int64_t nsv, double b);

// ---------------------------------------------------------------- Cascade SVM (L5)
// One native driver (csrc/cascade) for the classical tree (mpi_svm_main3.cpp) and the modified
// two-layer star (mpi_svm_main2.cpp) cascades; see cascade.h for the round semantics.
typedef struct svm_cascade_cfg {
  int32_t tree;            // 0 = star (modified two-layer), 1 = tree (classical, P a power of 2)
  int32_t max_rounds;      // 50 (mpi_svm_main3.cpp:544)
  svm_params params;
  int32_t log;             // rank 0 prints the reference's [rank 0] lines
  int32_t resume;          // start from <checkpoint_dir>/cascade_state.bin if present
  const char* checkpoint_dir;  // NULL or "" = no per-round checkpoint
  double comm_timeout_s;   // deadline of one blocking exchange (<= 0: 600 s)
  int32_t fail_rank;       // fault injection: this rank fails at the start of fail_round (-1 = off):
  int32_t fail_round;      //   it throws, or with fail_stall_s > 0 it stops responding for that long
  double fail_stall_s;     //   (the others then hit comm_timeout_s)
  int32_t solver;          // every local / merge solve: 0 = the pairwise first-order SMO (the reference's
                           //   trajectory, default), 1 = the warm-started working-set decomposition
                           //   (device backend: decomp.hip; CPU backend: its oracle on the set's kernel
                           //   matrix), 2 = per solve: the decomposition for cold or small sets
                           //   (<= SVM_CASCADE_DECOMP_WARM_ROWS rows), the pairwise SMO for large warm ones
  int32_t reserved;
} svm_cascade_cfg;

#define SVM_CASCADE_SOLVE_COLS 14
#define SVM_CASCADE_DECOMP_WARM_ROWS 4096
// Result of a cascade fit (allocated by the library, release with svm_cascade_free).
typedef struct svm_cascade_out {
  int32_t world, rank, rounds, converged;
  double b;
  double train_ms;         // max over the ranks this call drove (after the data distribution)
  int64_t d, n_sv;
  int64_t* ids;            // n_sv global sample ids of the final SVs (rank 0's SV order)
  int32_t* y;              // n_sv labels
  double* alpha;           // n_sv alphas
  double* sv_rows;         // n_sv x d scaled rows
  double* mn;              // d: global column min / max the rows were scaled with
  double* mx;
  int64_t n_hist;          // rounds recorded on rank 0
  int64_t* sv_history;     // n_hist global SV counts
  double* round_ms;        // n_hist round wall times (rank 0)
  int64_t n_merged;
  int64_t* merged_history; // star: rank 0's merged set sizes
  int64_t n_solves;
  double* solves;          // n_solves x SVM_CASCADE_SOLVE_COLS: rank, round, layer (star 0 local /
                           //   -1 merge, tree step), rows, SMO iterations, ms, b, stop reason, of ms
                           //   the kernel matrix, skipped (warm start already optimal), row cache
                           //   (solved on kernel rows computed on demand: the Gram did not fit),
                           //   solo ms (device time alone, serial-solve rehearsals; < 0 otherwise),
                           //   solver (0 pairwise SMO, 1 decomposition), decomposition outer iterations (0 pairwise)
  int64_t n_ranks;
  double* rank_train_ms;   // train_ms of each rank this call drove
  char transport[16];
  char backend[16];
  // Lowest driven rank's wall time per driver phase (cascade.h CascadePhase): upload, scale, bcast,
  // assemble, solve, select, gather, sendrecv, checkpoint, final, setup.
  double phase_ms[11];
} svm_cascade_out;

SVM_API void svm_cascade_default_cfg(svm_cascade_cfg* c);
// world thread-ranks in this process on the CPU oracle backend, loopback transport; rows X (n x d,
// float64) are partitioned into contiguous chunks of ceil(n / world) with global ids.
// Returns NULL on failure (svm_last_error(); a failed rank makes every rank leave its exchange).
SVM_API svm_cascade_out* svm_cascade_fit_cpu(const double* X, const int32_t* y, int64_t n, int64_t d,
                                             int32_t world, const svm_cascade_cfg* cfg);
SVM_API void svm_cascade_free(svm_cascade_out* o);

// One cascade rank per process on the CPU oracle backend, exchanging through caller-supplied
// collectives (e.g. a torch.distributed gloo group: svm355.parallel.hostcomm) -- the CPU twin of
// the per-process RCCL rank, svmd_cascade_rank_fit.  Buffers are host memory; every callback
// returns 0 on success.  gather's recv is NULL on non-root ranks (root: world * bytes, rank order).
typedef struct svm_host_comm {
  void* ctx;
  int32_t rank, world;
  int (*bcast)(void* ctx, void* buf, int64_t bytes, int32_t root);
  int (*allgather)(void* ctx, const void* send, int64_t bytes, void* recv);  // recv: world * bytes
  int (*allreduce_f64)(void* ctx, double* buf, int64_t n, int32_t op);       // op 0 = min, 1 = max
  int (*gather)(void* ctx, const void* send, int64_t bytes, void* recv, int32_t root);
  int (*send)(void* ctx, const void* buf, int64_t bytes, int32_t peer);
  int (*recv)(void* ctx, void* buf, int64_t bytes, int32_t peer);
  int (*barrier)(void* ctx);
} svm_host_comm;
// This process's rank trains on its partition (n_part x d float64 host rows, labels, global ids).
SVM_API svm_cascade_out* svm_cascade_rank_fit_cpu(const svm_host_comm* comm, const double* X, const int32_t* y,
                                                  const int64_t* ids, int64_t n_part, int64_t d, int64_t n_total,
                                                  const svm_cascade_cfg* cfg);

// The distributed form of svm_decomp_train_gram (decomp.hip's world > 1 solve on the CPU oracle): this
// process's rank owns 1/world of the selection blocks and of f, and the ranks all-gather their
// candidate records once per outer iteration through `comm`; every rank passes the whole K and gets the
// whole alpha (a replica).  For world dividing 8 the trajectory is svm_decomp_train_gram's bit for bit.
// Fault injection: SVM355_DECOMP_FAIL_RANK / SVM355_DECOMP_FAIL_OUTER (that rank fails at that outer
// iteration; its peers leave their exchange with an error).
SVM_API int svm_decomp_rank_train_gram(const svm_host_comm* comm, const double* K, int64_t ldk, const int32_t* y,
                                       int64_t n, double* alpha, int32_t warm, const svm_params* p, int32_t q,
                                       double tau_frac, int32_t inner_wss, svm_result* r, int64_t* stats);
// The same over `world` thread-ranks of this process (strict loopback transport); alpha, r and stats
// are rank 0's, and every rank's alpha replica must equal it.
SVM_API int svm_decomp_group_train_gram(int32_t world, const double* K, int64_t ldk, const int32_t* y, int64_t n,
                                        double* alpha, int32_t warm, const svm_params* p, int32_t q, double tau_frac,
                                        int32_t inner_wss, svm_result* r, int64_t* stats, double comm_timeout_s);

// Crash evidence (opt-in; Python: SVM355_CRASH_MAPS=<path>, "{pid}" replaced by the process id): on
// SIGSEGV / SIGBUS / SIGILL / SIGFPE / SIGABRT append the signal, faulting address, PC, a raw backtrace
// and /proc/self/maps to `path` (async-signal-safe calls only), then chain to the previous handler.
SVM_API int svm_crash_handler_install(const char* path);

// Transport exerciser (tests): world CPU-backend thread-ranks over a loopback group (strict = RCCL
// rules: matched collectives, rendezvous sends, deadlock detection) run `script` (exercise.cpp) with
// checked payloads.  SVM_OK, or an error naming the ranks / op within timeout_s.
SVM_API int svm_loopback_exercise(int32_t world, const char* script, int32_t strict, double timeout_s,
                                  double* elapsed_s);
// The preflight op list the device groups run on their RCCL communicators (needs cap bytes; returns
// the size needed when cap is too small, else 0).
SVM_API int svm_preflight_script(int32_t world, int64_t bulk_bytes, char* out, int64_t cap);

#ifdef __cplusplus
}
#endif
