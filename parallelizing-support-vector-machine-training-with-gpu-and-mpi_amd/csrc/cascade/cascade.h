// Native Cascade SVM: ONE driver for both topologies of the reference, any backend, any transport.
//
//   tree  classical Cascade, mpi_svm_main3.cpp:565-828 (power-of-two P; layers step = 1, 2, ..., P)
//   star  modified two-layer Cascade, mpi_svm_main2.cpp:439-769 (any P; gather to rank 0, whose
//         merge keeps its own alphas and resets the workers' to 0, :600-601)
//
// The driver (run_cascade, cascade.cpp) is written once against two interfaces:
//   Backend    where rows live and solves run: CpuBackend (the C++ oracle, host memory; in
//              libsvm355_core) or the gfx950 device backend (HBM, MFMA Gram + device SMO; in
//              libsvm355_hip).  An SV set is a structure of arrays in backend memory.
//   Transport  the reference's MPI call sites as a handful of collectives: LoopbackTransport
//              (thread ranks of one process, host-staged; in libsvm355_core) or RcclTransport
//              (RCCL over xGMI, one communicator per GPU; in libsvm355_hip).
// so the CPU tests exercise exactly the code the 8-GPU run executes.
//
// Failure handling (the reference's MPI_Abort, M3 :420-428, :450-454): every blocking
// wait of a transport polls a shared AbortToken and a deadline; the first rank that fails raises the
// token, the others leave their collective with CascadeAborted, and the RCCL communicators are
// aborted (ncclCommAbort) before the error is reported.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "svm355.h"

namespace svm355 {

struct CascadeError : std::runtime_error {  // configuration / data errors (no peer involved)
  using std::runtime_error::runtime_error;
};
struct TransportError : std::runtime_error {  // a collective failed or timed out
  using std::runtime_error::runtime_error;
};
struct CascadeAborted : std::runtime_error {  // another rank failed first
  using std::runtime_error::runtime_error;
};

// Shared by the ranks of one process: raised by the first failing rank.
class AbortToken {
 public:
  bool raised() const { return flag_.load(std::memory_order_acquire); }
  void raise(const std::string& why) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!flag_.load(std::memory_order_relaxed)) why_ = why;
    flag_.store(true, std::memory_order_release);
  }
  std::string why() const {
    std::lock_guard<std::mutex> lk(mu_);
    return why_;
  }

 private:
  std::atomic<bool> flag_{false};
  mutable std::mutex mu_;
  std::string why_;
};

// Deadline of one blocking transport wait.
struct WaitPolicy {
  std::shared_ptr<AbortToken> token;  // may be null (multi-process ranks: deadline only)
  double timeout_s = 600.0;
  // Throws CascadeAborted / TransportError when the token is raised or the deadline has passed.
  void check(std::chrono::steady_clock::time_point start, const char* what) const;
};

// ------------------------------------------------------------------------------------ backends
// Memory owned by a backend (device memory for the HIP backend, host memory for the CPU one).
class Backend;
class Buf {
 public:
  Buf() = default;
  explicit Buf(Backend* b) : b_(b) {}
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  Buf(Buf&& o) noexcept { *this = std::move(o); }
  Buf& operator=(Buf&& o) noexcept;
  ~Buf() { reset(); }
  void reset();
  void ensure(int64_t bytes);  // grow-only; contents are not preserved when it grows
  void* release();             // hand the allocation to the caller (Backend::free it)
  void* get() const { return p_; }
  template <class T>
  T* as() const {
    return static_cast<T*>(p_);
  }
  int64_t bytes() const { return n_; }

 private:
  Backend* b_ = nullptr;
  void* p_ = nullptr;
  int64_t n_ = 0;
};

// SV set in backend memory (structure of arrays) + a host mirror of the global ids, which the
// ID de-duplication and the convergence test run on.
struct DSet {
  Buf X;   // k x ld scaled rows (zero padded)
  Buf y;   // k int32 +-1
  Buf a;   // k double alphas
  Buf id;  // k int64 global sample ids
  int64_t k = 0;
  std::vector<int64_t> ids;  // host copy of id
};

// One source segment of DSet assembly: rows idx (nullptr = all, in order) of a set or of a packed
// record buffer [row | y | alpha | id] (width ld + 3 doubles).
struct Segment {
  const DSet* set = nullptr;
  const double* rec = nullptr;  // backend memory
  int64_t rec_rows = 0;
  const int64_t* rec_ids = nullptr;  // host ids of the records
  const std::vector<int64_t>* idx = nullptr;
  bool zero_alpha = false;
  // Optional backend-memory copy of *idx (already there, e.g. from select_svs): assemble uses it
  // instead of staging idx again.
  const int64_t* idx_dev = nullptr;
  int64_t rows() const { return idx ? int64_t(idx->size()) : (set ? set->k : rec_rows); }
};

struct SolveStats {
  int64_t iterations = 0;
  double b = 0.0;
  int32_t stop = 0;
  double gram_ms = 0.0;
  bool row_cache = false;  // solved on the HBM row cache (the k x k Gram did not fit)
  int32_t solver = 0;      // the solver that ran: 0 pairwise SMO, 1 working-set decomposition
  int64_t outer = 0;       // decomposition: outer iterations (working sets solved)
};

class Backend {
 public:
  virtual ~Backend() = default;
  virtual const char* name() const = 0;
  virtual int64_t ld(int64_t d) const = 0;  // row stride of stored rows
  virtual void* alloc(int64_t bytes) = 0;
  virtual void free(void* p) = 0;
  virtual void h2d(void* dst, const void* src, int64_t bytes) = 0;  // synchronous
  virtual void d2h(void* dst, const void* src, int64_t bytes) = 0;  // synchronous
  virtual void sync() = 0;
  // Host rows (float64, or uint8 pixels when u8) -> stored rows (n x ld).
  virtual void upload_rows(const void* X, bool u8, int64_t n, int64_t d, double* dst) = 0;
  // Column min/max of n stored rows (n == 0: +inf / -inf); mn/mx are backend buffers of d.
  virtual void minmax(const double* X, int64_t n, int64_t d, double* mn, double* mx) = 0;
  // In-place min-max scaling with the range < 1e-12 -> 1 rule; mn/mx are backend buffers.
  virtual void scale(double* X, int64_t n, int64_t d, const double* mn, const double* mx) = 0;
  // dst rows [off, off + seg.rows()) from seg (alphas zeroed on request).
  virtual void assemble(const Segment& seg, int64_t ld, DSet& dst, int64_t off) = 0;
  // rec[i] = [row | y | alpha | id], i < S.k (rec holds cap >= S.k records).
  virtual void pack(const DSet& S, int64_t ld, double* rec) = 0;
  // ids[i] = record i's id, i < k.
  virtual void record_ids(const double* rec, int64_t k, int64_t ld, int64_t* ids_host) = 0;
  // Several record buffers at once (one host round trip on a device backend): ids_host[s][i] =
  // record i's id of source s, i < ks[s].
  virtual void record_ids_batch(const std::vector<const double*>& recs, const std::vector<int64_t>& ks, int64_t ld,
                                const std::vector<int64_t*>& ids_host) {
    for (size_t s = 0; s < recs.size(); ++s)
      if (ks[s]) record_ids(recs[s], ks[s], ld, ids_host[s]);
  }
  // Ascending indices of S's rows with alpha > tol (SV extraction, main3.cpp:297-304) into keep;
  // *keep_dev = a backend-memory copy of them valid until the next call (nullptr: none, assemble
  // stages keep itself).  Default: alphas read back to the host.
  virtual void select_svs(const DSet& S, double tol, std::vector<int64_t>* keep, const int64_t** keep_dev) {
    std::vector<double> a(static_cast<size_t>(S.k));
    if (S.k) d2h(a.data(), S.a.get(), S.k * 8);
    keep->clear();
    for (int64_t i = 0; i < S.k; ++i)
      if (a[size_t(i)] > tol) keep->push_back(i);
    *keep_dev = nullptr;
  }
  // Warm-start solve on S (SMO_train(..., init=false), mpi_svm_main3.cpp:155-290): alphas in S.a are
  // updated in place.  mn_h/mx_h: the global scaling statistics (host, d values).  solver: 0 the
  // pairwise SMO, 1 the working-set decomposition (CascadeConfig::solver; the stats say which ran).
  // warm_rows: S's leading rows that carry the warm alphas (0: a cold start).
  virtual SolveStats solve(DSet& S, int64_t d, const svm_params& p, const double* mn_h, const double* mx_h,
                           int solver, int64_t warm_rows) = 0;
  // True when the warm start of S (rows [0, nz) carry every nonzero alpha) provably meets the stop
  // test b_low <= b_high + 2 tau already -- i.e. the solve would end at its first selection without
  // an update -- checked from a cross-kernel K(S, S[0:nz]) only, before any Gram work.  The margin
  // covers the check's own rounding, so a true answer never changes a result.  Default: never.
  virtual bool warm_start_converged(DSet& S, int64_t nz, int64_t d, const svm_params& p, const double* mn_h,
                                    const double* mx_h) {
    return false;
  }
  // Device time of the solve work since the last call, measured with the device to this rank alone
  // (HIP backend with SVM355_CASCADE_SERIAL_SOLVES=1: a one-GPU rehearsal of P ranks runs their
  // solves one at a time, so each is timed as it would run on its own GPU); < 0 when not measured.
  virtual double take_solo_ms() { return -1.0; }
  virtual void trace_push(const char*) {}  // roctx ranges (HIP backend)
  virtual void trace_pop() {}
};

// ---------------------------------------------------------------------------------- transports
// Every buffer argument is backend memory of the calling rank; each call returns once its data is
// complete (payloads are a few MB per round between solves of milliseconds).
//
// | reference call site                                   | Transport method                       |
// |-------------------------------------------------------|----------------------------------------|
// | MPI_Bcast n_features / n_total, SV count, converged   | bcast_i64                              |
// | MPI_Bcast min / max (M3 :534-535)                     | allreduce_min / allreduce_max of the   |
// |                                                       |   local column statistics              |
// | MPI_Bcast X_sv, Y_sv, alpha_sv, ID_sv (M3 :598-601)   | bcast of ONE packed SV buffer          |
// | star MPI_Send/Recv to rank 0 (M2 :578-607, 748-760)   | allgather_i64 (counts) + gather of     |
// |                                                       |   max-count-padded packed buffers      |
// | tree MPI_Send/Recv pairs (M3 :689-716)                | send_i64 / send + recv_i64 / recv      |
// | MPI_Abort (M3 :426, :453)                             | abort()                                |
class Transport {
 public:
  virtual ~Transport() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  virtual int64_t bcast_i64(int64_t v, int root) = 0;
  virtual std::vector<int64_t> allgather_i64(int64_t v) = 0;
  virtual void allreduce_min(double* buf, int64_t n) = 0;
  virtual void allreduce_max(double* buf, int64_t n) = 0;
  virtual void bcast(void* buf, int64_t bytes, int root) = 0;
  // Every rank sends `bytes` from send; root receives world * bytes into recv (rank order).
  virtual void gather(const void* send, int64_t bytes, void* recv, int root) = 0;
  // All-gather of `bytes` from every rank into recv (world * bytes, rank-major), e.g. the distributed
  // decomposition SMO's candidate records.  Default: a gather to rank 0, then a broadcast of it.
  virtual void allgather(const void* send, int64_t bytes, void* recv) {
    gather(send, bytes, recv, 0);
    bcast(recv, bytes * world(), 0);
  }
  // The all-gather enqueued on the rank's stream without waiting for it; the caller then waits
  // with stream_wait.  Transports that exchange through the host complete it here.
  virtual void allgather_async(const void* send, int64_t bytes, void* recv) { allgather(send, bytes, recv); }
  // Wait for the rank's stream under the transport's deadline / abort policy.  false: this transport
  // has no stream of its own to poll (the caller synchronises its stream itself).
  virtual bool stream_wait(const char* what) {
    (void)what;
    return false;
  }
  // The same for a recorded event (a hipEvent_t) of the rank's stream.
  virtual bool event_wait(void* event, const char* what) {
    (void)event;
    (void)what;
    return false;
  }
  virtual void send_i64(int64_t v, int peer) = 0;
  virtual int64_t recv_i64(int peer) = 0;
  virtual void send(const void* buf, int64_t bytes, int peer) = 0;
  virtual void recv(void* buf, int64_t bytes, int peer) = 0;
  virtual void barrier() = 0;
  virtual void abort() {}  // release the communicator after a failure (ncclCommAbort)
  virtual const char* name() const = 0;
};

// P thread-ranks of one process exchanging through host memory (staged with the backend's copies),
// so any P runs on one GPU (RCCL refuses two ranks on one device) or on the CPU.
//
// Strict mode (the default) holds every call sequence to RCCL's rules, so a sequence that would
// deadlock or mismatch over RCCL fails here too, with both ranks named:
//   * collectives: every rank records (op, root, bytes) before the first barrier of the call and
//     every rank compares all records after it -- any difference throws TransportError on every rank;
//   * send is a rendezvous (ncclSend completes once matched): it returns only when the peer's recv
//     has taken the message, and a byte-count mismatch fails on both sides;
//   * every wait checks the wait-for graph of the blocked ranks (a collective waits for the ranks
//     that have not arrived, send / recv for the peer): a cycle is a deadlock and throws at once
//     instead of at the deadline.
// Non-strict mode (strict = false) keeps the old mailbox semantics (send returns after posting).
class LoopbackGroup {
 public:
  enum OpKind : int { kIdle = 0, kBcastI64, kAllgatherI64, kAllreduceMin, kAllreduceMax, kBcast, kGather, kBarrier,
                      kSend, kRecv };
  struct OpDesc {
    int kind = kIdle;
    int root = -1;       // collectives with a root
    int64_t bytes = -1;  // payload per rank (-1: not part of the op's signature)
    int peer = -1;       // send / recv
  };
  LoopbackGroup(int world, WaitPolicy wp, bool strict = true);
  int world() const { return world_; }
  bool strict() const { return strict_; }
  // One collective call of `rank`: records op, waits for every rank (first barrier), checks the
  // records (strict), then runs `between` (reads of the peers' slots), and waits again.
  void collective(int rank, const OpDesc& op, const std::function<void()>& between);
  void arrive_and_wait(int rank = -1);  // reusable (generation-counted) barrier, honours the wait policy
  std::vector<char>& slot(int r) { return slots_[size_t(r)]; }
  // Point-to-point: post enqueues (strict: and waits until the receiver took it); take dequeues the
  // next message src -> dst, checking its size against `expect` (< 0: any size).
  void post(int src, int dst, std::vector<char> msg);
  std::vector<char> take(int src, int dst, int64_t expect = -1);
  const WaitPolicy& policy() const { return wp_; }
  static const char* op_name(int kind);

 private:
  struct Msg {
    std::vector<char> data;
    uint64_t seq = 0;
  };
  struct RankState {
    OpDesc op;         // the call the rank is inside (kIdle: none)
    uint64_t gen = 0;  // collectives: barrier generation it waits on
    uint64_t seq = 0;  // send: sequence number of its message on the channel
  };
  void wait_until(std::unique_lock<std::mutex>& lk, int rank, const char* what, const std::function<bool()>& done);
  bool blocked(int r) const;                  // under mu_
  std::vector<int> waits_for(int r) const;    // under mu_
  std::string deadlock_cycle(int r) const;    // under mu_: "" or a description of the cycle through r
  std::string describe(int r) const;          // under mu_
  int world_;
  WaitPolicy wp_;
  bool strict_;
  std::mutex mu_;
  std::condition_variable cv_;
  int waiting_ = 0;
  uint64_t gen_ = 0;
  std::vector<std::vector<char>> slots_;
  std::vector<std::deque<Msg>> mail_;  // [src * world + dst] FIFO
  std::vector<uint64_t> sent_, taken_;  // per channel: messages posted / taken
  std::vector<int64_t> rejected_;       // per channel: seq + 1 of a message the receiver refused (size)
  std::vector<RankState> st_;
  std::vector<OpDesc> coll_;            // per rank: the descriptor of its current collective
  std::string mismatch_;                // strict: the first rank-pair mismatch of the current generation
};

class LoopbackTransport : public Transport {
 public:
  LoopbackTransport(std::shared_ptr<LoopbackGroup> g, int rank, Backend* mem) : g_(std::move(g)), rank_(rank), mem_(mem) {}
  int rank() const override { return rank_; }
  int world() const override { return g_->world(); }
  int64_t bcast_i64(int64_t v, int root) override;
  std::vector<int64_t> allgather_i64(int64_t v) override;
  void allreduce_min(double* buf, int64_t n) override { allreduce(buf, n, true); }
  void allreduce_max(double* buf, int64_t n) override { allreduce(buf, n, false); }
  void bcast(void* buf, int64_t bytes, int root) override;
  void gather(const void* send, int64_t bytes, void* recv, int root) override;
  void send_i64(int64_t v, int peer) override;
  int64_t recv_i64(int peer) override;
  void send(const void* buf, int64_t bytes, int peer) override;
  void recv(void* buf, int64_t bytes, int peer) override;
  void barrier() override;
  const char* name() const override { return "loopback"; }

 private:
  void to_host(std::vector<char>& dst, const void* src, int64_t bytes);
  void to_backend(void* dst, const std::vector<char>& src, int64_t bytes);
  void allreduce(double* buf, int64_t n, bool is_min);
  std::shared_ptr<LoopbackGroup> g_;
  int rank_;
  Backend* mem_;
};

// ------------------------------------------------------------------------------------ the driver
struct CascadeConfig {
  bool tree = false;    // false = star (modified two-layer)
  int max_rounds = 50;  // mpi_svm_main3.cpp:544, mpi_svm_main2.cpp:428
  svm_params params{};  // C, gamma, tau, eps, sv_tol, max_iter, n_threads
  bool log = true;      // rank 0 prints the reference's per-round lines
  // Per-round checkpoint: rank 0 writes <checkpoint_dir>/cascade_state.bin after every
  // round (global SV set with alphas, b, next round); resume = start from that file if present.
  std::string checkpoint_dir;
  bool resume = false;
  // Fault injection (tests): rank fail_rank throws at the start of round fail_round (-1 = off), or
  // with fail_stall_s > 0 stops responding for that long (its peers' exchanges hit the deadline).
  int fail_rank = -1, fail_round = -1;
  double fail_stall_s = 0.0;
  int solver = 0;  // svm_cascade_cfg.solver: 0 pairwise SMO, 1 working-set decomposition, 2 per solve
};

// svm_cascade_cfg.solver = 2: the solver of one solve.  Measured at 60k (profiles/r4_cascade_decomp_rehearsal.txt):
// the decomposition is 1.4-2.2x faster on cold and small warm sets (round-0 locals, merges), 4-6x slower on
// large warm-started sets (later-round locals of P <= 4: hundreds of working sets of ~20-90 pair updates).
inline int cascade_solver_for(int solver, int64_t k, int64_t warm_rows) {
  if (solver != 2) return solver;
  return (warm_rows == 0 || k <= SVM_CASCADE_DECOMP_WARM_ROWS) ? 1 : 0;
}

// cascade_state.bin layout (little-endian): char magic[8] = "SVM355C3"; int32 topology (0 star,
// 1 tree); int32 reserved; int64 next_round; double b; int64 d; int64 k; uint64 fingerprint of the
// training set (FNV-1a over n, the global column min / max and the ranks' hashes of their rows, labels
// and global ids, when a checkpoint directory is set); then k records of d + 3 doubles
// [scaled row (d) | y | alpha | global id] (backend independent).
constexpr char kCheckpointMagic[9] = "SVM355C3";

struct SolveLog {
  int rank = 0, round = 0;
  int layer = 0;  // star: 0 = local, -1 = rank-0 merge; tree: the layer's step (1, 2, ..., P)
  int64_t rows = 0, iterations = 0;
  double ms = 0.0, b = 0.0;
  int32_t stop = 0;
  double gram_ms = 0.0;  // of ms: the kernel matrix (device backend)
  bool skipped = false;  // warm start already met the stop test (Backend::warm_start_converged)
  bool row_cache = false;  // SolveStats::row_cache
  double solo_ms = -1.0;   // Backend::take_solo_ms (skip check + solve), < 0 = not measured
  int32_t solver = 0;      // SolveStats::solver
  int64_t outer = 0;       // SolveStats::outer
};

// Wall time of this rank per driver phase (host clock; with SVM355_CASCADE_PROFILE=1 every phase
// ends with a backend sync, so asynchronous device work is charged to the phase that issued it).
enum CascadePhase {
  kPhUpload = 0,   // partition H2D (before the timed region)
  kPhScale,        // local min/max, all-reduce, scaling
  kPhBcast,        // global SV broadcast (pack, collective, record ids, assembly)
  kPhAssemble,     // training-set assembly: ID de-duplication + row gathers
  kPhSolve,        // warm-start SMO solves (Gram + SMO)
  kPhSelect,       // alpha read-back + SV extraction
  kPhGather,       // star: counts + padded gather to rank 0
  kPhSendRecv,     // tree: pairwise exchanges
  kPhCheckpoint,   // per-round state file
  kPhFinal,        // final b / SV broadcast and the host copy of the model
  kPhSetup,        // driver entry to the start of the timed region, without the upload
  kNumPhases
};

struct CascadeOutput {
  double phase_ms[kNumPhases] = {};
  // Final global SV set (every rank holds it after the final broadcast).
  std::vector<int64_t> ids;
  std::vector<int32_t> y;
  std::vector<double> alpha;
  DSet final_set;  // the same rows in backend memory (ld stride)
  int64_t d = 0, ld = 0;
  double b = 0.0;
  int rounds = 0;
  bool converged = false;
  std::vector<int64_t> sv_history, merged_history;  // rank 0
  std::vector<double> round_ms;                     // rank 0
  double train_ms = 0.0;                            // this rank, after the data distribution
  std::vector<double> mn, mx;  // global column min / max the rows were scaled with
  std::vector<SolveLog> solves;  // this rank's solves
};

// Train on this rank's partition: X (n_part x d host rows, float64 or uint8 when u8), labels +-1,
// global sample ids.  Throws CascadeError / TransportError / CascadeAborted.
CascadeOutput run_cascade(Transport& t, Backend& B, const void* X, bool u8, const int32_t* y, const int64_t* ids,
                          int64_t n_part, int64_t d, int64_t n_total, const CascadeConfig& cfg);

// Contiguous chunks of ceil(N/P) rows (mpi_svm_main3.cpp:464-518).
inline void partition_bounds(int64_t n, int P, int r, int64_t* lo, int64_t* hi) {
  const int64_t chunk = (n + P - 1) / P;
  *lo = std::min<int64_t>(n, int64_t(r) * chunk);
  *hi = std::min<int64_t>(n, *lo + chunk);
}

// One thread per rank: fn(rank) runs the rank's cascade; the first exception raises the token
// (the others leave their collectives), every rank's transport is aborted, and the first error is
// rethrown as CascadeError with the rank that failed.  Returns when every thread has ended.
void run_rank_threads(int P, const std::shared_ptr<AbortToken>& token, const std::function<void(int)>& fn,
                      const std::function<void(int)>& on_abort);

// Persistent rank threads (one per rank, kept by a device group between fits, so no fit pays
// thread creation / per-thread runtime set-up and teardown).  run() has run_rank_threads semantics.
class RankPool {
 public:
  explicit RankPool(int P);
  ~RankPool();
  RankPool(const RankPool&) = delete;
  RankPool& operator=(const RankPool&) = delete;
  int size() const { return P_; }
  void run(const std::shared_ptr<AbortToken>& token, const std::function<void(int)>& fn,
           const std::function<void(int)>& on_abort);

 private:
  void loop(int r);
  int P_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
  const std::function<void(int)>* job_ = nullptr;
  std::shared_ptr<AbortToken> token_;
};

std::unique_ptr<Backend> make_cpu_backend();

}  // namespace svm355
