// Native Cascade SVM driver (see cascade.h): the round logic of mpi_svm_main2.cpp (star) and
// mpi_svm_main3.cpp (tree), written once against the Backend / Transport interfaces.
//
// SV sets live in backend memory as structures of arrays; an exchange packs a set into ONE record
// buffer k x (ld + 3) doubles [row | y | alpha | id] (ids < 2^53 and +-1 labels are exact in
// float64), so every exchange is a count plus one bulk transfer.  Only the global ids (for the ID
// de-duplication of M3 :629-655 / M2 :474-502, 578-607 and the ID-set convergence test, M3 :725-743)
// and the solved alphas (for the alpha > sv_tol selection) cross to the host.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <numeric>
#include <thread>
#include <unordered_set>
#include <utility>

#include "cascade.h"

namespace svm355 {

// ---------------------------------------------------------------------------------- wait policy
void WaitPolicy::check(std::chrono::steady_clock::time_point start, const char* what) const {
  if (token && token->raised()) throw CascadeAborted(std::string("left ") + what + ": " + token->why());
  if (timeout_s > 0) {
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
    if (s > timeout_s) {
      char buf[64];
      snprintf(buf, sizeof(buf), "%.1f", timeout_s);
      throw TransportError(std::string(what) + ": no progress for " + buf + " s (a peer rank stopped responding)");
    }
  }
}

// ----------------------------------------------------------------------------------------- Buf
Buf& Buf::operator=(Buf&& o) noexcept {
  if (this != &o) {
    reset();
    b_ = o.b_;
    p_ = o.p_;
    n_ = o.n_;
    o.p_ = nullptr;
    o.n_ = 0;
  }
  return *this;
}

void Buf::reset() {
  if (p_ && b_) b_->free(p_);
  p_ = nullptr;
  n_ = 0;
}

void Buf::ensure(int64_t bytes) {
  if (p_ && bytes <= n_) return;
  reset();
  n_ = std::max<int64_t>(bytes, 8);
  p_ = b_->alloc(n_);
}

void* Buf::release() {
  void* q = p_;
  p_ = nullptr;
  n_ = 0;
  return q;
}

// -------------------------------------------------------------------------------- rank threads
void run_rank_threads(int P, const std::shared_ptr<AbortToken>& token, const std::function<void(int)>& fn,
                      const std::function<void(int)>& on_abort) {
  std::vector<std::thread> th;
  th.reserve(size_t(P));
  for (int r = 0; r < P; ++r)
    th.emplace_back([&, r] {
      try {
        fn(r);
      } catch (const CascadeAborted&) {
        // another rank failed first; its message is the one reported
      } catch (const std::exception& e) {
        token->raise("rank " + std::to_string(r) + ": " + e.what());
      }
    });
  for (auto& t : th) t.join();
  if (token->raised()) {
    for (int r = 0; r < P; ++r) on_abort(r);
    throw CascadeError(token->why());
  }
}

RankPool::RankPool(int P) : P_(P) {
  th_.reserve(size_t(P));
  for (int r = 0; r < P; ++r) th_.emplace_back([this, r] { loop(r); });
}

RankPool::~RankPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
    ++gen_;
  }
  cv_.notify_all();
  for (auto& t : th_) t.join();
}

void RankPool::loop(int r) {
  uint64_t seen = 0;
  for (;;) {
    const std::function<void(int)>* job;
    std::shared_ptr<AbortToken> token;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (stop_) return;
      job = job_;
      token = token_;
    }
    try {
      (*job)(r);
    } catch (const CascadeAborted&) {
    } catch (const std::exception& e) {
      token->raise("rank " + std::to_string(r) + ": " + e.what());
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
}

void RankPool::run(const std::shared_ptr<AbortToken>& token, const std::function<void(int)>& fn,
                   const std::function<void(int)>& on_abort) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    job_ = &fn;
    token_ = token;
    pending_ = P_;
    ++gen_;
  }
  cv_.notify_all();
  {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
    token_.reset();
  }
  if (token->raised()) {
    for (int r = 0; r < P_; ++r) on_abort(r);
    throw CascadeError(token->why());
  }
}

namespace {

using Clock = std::chrono::steady_clock;
double ms_between(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

struct Range {  // roctx range through the backend (rocprofv3 --marker-trace), SURVEY §5.1
  Backend& b;
  Range(Backend& be, const std::string& name) : b(be) { b.trace_push(name.c_str()); }
  ~Range() { b.trace_pop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

// Adds the scope's wall time to one CascadePhase accumulator (optionally after a backend sync).
struct PhaseTimer {
  Backend& b;
  double& acc;
  bool sync;
  Clock::time_point t0 = Clock::now();
  PhaseTimer(Backend& be, double& a, bool s) : b(be), acc(a), sync(s) {}
  ~PhaseTimer() {
    if (sync) {
      try {
        b.sync();
      } catch (...) {  // the next checked call reports the error
      }
    }
    acc += ms_between(t0, Clock::now());
  }
  PhaseTimer(const PhaseTimer&) = delete;
  PhaseTimer& operator=(const PhaseTimer&) = delete;
};

class Rank {
 public:
  Rank(Transport& t, Backend& B, int64_t d, const CascadeConfig& cfg)
      : t_(t), B_(B), d_(d), ld_(B.ld(d)), w_(B.ld(d) + 3), cfg_(cfg), pack_(&B), recv_(&B) {
    const char* e = getenv("SVM355_CASCADE_PROFILE");
    prof_ = e && atoi(e) != 0;
  }

  std::vector<double> mn_h, mx_h;
  std::vector<SolveLog> log;
  double phase[kNumPhases] = {};
  int64_t skipped = 0;  // solves whose warm start already met the stop test
  PhaseTimer timer(CascadePhase p) { return PhaseTimer(B_, phase[p], prof_); }

  DSet make(int64_t k) {
    DSet s;
    s.X = Buf(&B_);
    s.y = Buf(&B_);
    s.a = Buf(&B_);
    s.id = Buf(&B_);
    s.k = k;
    if (k) {
      s.X.ensure(k * ld_ * 8);
      s.y.ensure(k * 4);
      s.a.ensure(k * 8);
      s.id.ensure(k * 8);
    }
    s.ids.resize(size_t(k));
    return s;
  }

  // Concatenation of segments, in order (each one a single backend launch).
  DSet assemble(const std::vector<Segment>& segs) {
    int64_t k = 0;
    for (const Segment& s : segs) k += s.rows();
    DSet o = make(k);
    int64_t off = 0;
    for (const Segment& s : segs) {
      const int64_t m = s.rows();
      if (!m) continue;
      B_.assemble(s, ld_, o, off);
      const int64_t* src_ids = s.set ? s.set->ids.data() : s.rec_ids;
      for (int64_t i = 0; i < m; ++i) o.ids[size_t(off + i)] = src_ids[s.idx ? (*s.idx)[size_t(i)] : i];
      off += m;
    }
    return o;
  }

  DSet upload(const void* X, bool u8, const int32_t* y, const int64_t* ids, int64_t n) {
    auto tm = timer(kPhUpload);
    DSet s = make(n);
    if (n) {
      B_.upload_rows(X, u8, n, d_, s.X.as<double>());
      B_.h2d(s.y.get(), y, n * 4);
      const std::vector<double> z(size_t(n), 0.0);
      B_.h2d(s.a.get(), z.data(), n * 8);
      B_.h2d(s.id.get(), ids, n * 8);
      std::copy(ids, ids + n, s.ids.begin());
    }
    return s;
  }

  // Scale this rank's partition with the globally all-reduced column min / max (bitwise equal to
  // the reference's rank-0 min/max + MPI_Bcast, M3 :529-539).
  void scale_global(DSet& part) {
    auto tm = timer(kPhScale);
    Buf mn(&B_), mx(&B_);
    mn.ensure(d_ * 8);
    mx.ensure(d_ * 8);
    B_.minmax(part.X.as<double>(), part.k, d_, mn.as<double>(), mx.as<double>());
    t_.allreduce_min(mn.as<double>(), d_);
    t_.allreduce_max(mx.as<double>(), d_);
    if (part.k) B_.scale(part.X.as<double>(), part.k, d_, mn.as<double>(), mx.as<double>());
    mn_h.resize(size_t(d_));
    mx_h.resize(size_t(d_));
    B_.d2h(mn_h.data(), mn.get(), d_ * 8);
    B_.d2h(mx_h.data(), mx.get(), d_ * 8);
  }
  // The training set a checkpoint belongs to: FNV-1a over n, the global column bounds and every rank's
  // rows, labels and ids (rows_hash, combined in rank order; a resume on other data -- other rows with
  // the same bounds, or the same rows with another positive class -- would otherwise warm-start from
  // another problem's support vectors without a word).
  uint64_t data_fingerprint(int64_t n_total, uint64_t rows_hash) const {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&h](const void* p, size_t bytes) {
      const auto* c = static_cast<const unsigned char*>(p);
      for (size_t i = 0; i < bytes; ++i) h = (h ^ c[i]) * 1099511628211ull;
    };
    mix(&n_total, 8);
    mix(mn_h.data(), mn_h.size() * 8);
    mix(mx_h.data(), mx_h.size() * 8);
    mix(&rows_hash, 8);
    return h;
  }
  uint64_t fingerprint = 0;  // set by run_cascade after the global scaling

  // warm (alphas kept) U rows of extra whose id is not in warm (alpha = 0), extra order kept
  // (the seen_ids loops of mpi_svm_main3.cpp:629-655 / mpi_svm_main2.cpp:474-502).
  DSet merge_unseen(const DSet& warm, const DSet& extra) {
    auto tm = timer(kPhAssemble);
    if (warm.k == 0) return assemble({Segment{&extra, nullptr, 0, nullptr, nullptr, true}});
    const std::unordered_set<int64_t> seen(warm.ids.begin(), warm.ids.end());
    std::vector<int64_t> keep;
    keep.reserve(size_t(extra.k));
    for (int64_t i = 0; i < extra.k; ++i)
      if (!seen.count(extra.ids[size_t(i)])) keep.push_back(i);
    return assemble({Segment{&warm, nullptr, 0, nullptr, nullptr, false},
                     Segment{&extra, nullptr, 0, nullptr, &keep, true}});
  }

  // Warm-start SMO on S; returns (its SVs with alpha > sv_tol, in S order, b).  warm_rows: S's
  // leading rows that carry the warm alphas; skippable: the solve's b is not part of the model, so
  // a warm start that provably meets the stop test may skip the solve (Backend::warm_start_converged:
  // the solve would have stopped at its first selection with the same alphas).
  std::pair<DSet, double> solve(DSet& S, int rnd, int layer, int64_t warm_rows = 0, bool skippable = false) {
    if (S.k == 0) return {make(0), 0.0};
    Range tr(B_, "cascade:solve");
    const auto t0 = Clock::now();
    SolveStats st;
    bool skipped_now = false;
    {
      auto tm = timer(kPhSolve);
      if (skippable && warm_rows > 0 &&
          B_.warm_start_converged(S, warm_rows, d_, cfg_.params, mn_h.data(), mx_h.data())) {
        st.iterations = 1;  // what the solve reports when it stops at its first selection
        st.stop = SVM_STOP_CONVERGED;
        st.b = 0.0;         // not part of the model (skippable)
        ++skipped;
        skipped_now = true;
      } else {
        st = B_.solve(S, d_, cfg_.params, mn_h.data(), mx_h.data(), cascade_solver_for(cfg_.solver, S.k, warm_rows),
                      warm_rows);
      }
    }
    auto tm = timer(kPhSelect);
    std::vector<int64_t> keep;
    const int64_t* keep_dev = nullptr;
    B_.select_svs(S, cfg_.params.sv_tol, &keep, &keep_dev);
    Segment seg{&S, nullptr, 0, nullptr, &keep, false};
    seg.idx_dev = keep_dev;
    DSet out = assemble({seg});
    log.push_back(
        SolveLog{t_.rank(), rnd, layer, S.k, st.iterations, ms_between(t0, Clock::now()), st.b, st.stop, st.gram_ms,
                              skipped_now, st.row_cache, B_.take_solo_ms(),
                              skipped_now ? cascade_solver_for(cfg_.solver, S.k, warm_rows) : st.solver,
                              st.outer});
    return {std::move(out), st.b};
  }

  // ---- exchanges
  DSet bcast_set(const DSet& G) {  // G meaningful on rank 0
    Range tr(B_, "cascade:bcast_svs");
    auto tm = timer(kPhBcast);
    const bool root = t_.rank() == 0;
    const int64_t k = t_.bcast_i64(root ? G.k : 0, 0);
    pack_.ensure(std::max<int64_t>(k, 1) * w_ * 8);
    if (root && k) B_.pack(G, ld_, pack_.as<double>());
    if (k) t_.bcast(pack_.get(), k * w_ * 8, 0);
    std::vector<int64_t> ids(static_cast<size_t>(k));
    if (root)
      ids = G.ids;
    else if (k)
      B_.record_ids(pack_.as<double>(), k, ld_, ids.data());
    Segment s;
    s.rec = pack_.as<double>();
    s.rec_rows = k;
    s.rec_ids = ids.data();
    return assemble({s});
  }

  // Star: local SV sets to rank 0 (counts all-gathered, max-count-padded gather, source order).
  struct Gathered {
    std::vector<int64_t> counts;
    int64_t kmax = 0;
    std::vector<std::vector<int64_t>> ids;  // rank 0: host ids of every source
  };
  Gathered gather_sets(const DSet& local) {
    Range tr(B_, "cascade:gather_svs");
    auto tm = timer(kPhGather);
    Gathered g;
    g.counts = t_.allgather_i64(local.k);
    g.kmax = *std::max_element(g.counts.begin(), g.counts.end());
    if (t_.rank() == 0) g.ids.resize(size_t(t_.world()));  // one (possibly empty) id list per source
    if (g.kmax == 0) return g;  // no rank has a support vector (e.g. every partition holds one class)
    pack_.ensure(g.kmax * w_ * 8);
    if (local.k) B_.pack(local, ld_, pack_.as<double>());
    const int64_t bytes = g.kmax * w_ * 8;
    const bool root = t_.rank() == 0;
    if (root) recv_.ensure(bytes * t_.world());
    t_.gather(pack_.get(), bytes, root ? recv_.get() : nullptr, 0);
    if (root) {
      std::vector<const double*> recs;
      std::vector<int64_t> ks;
      std::vector<int64_t*> outs;
      for (int r = 1; r < t_.world(); ++r) {
        g.ids[size_t(r)].resize(size_t(g.counts[size_t(r)]));
        recs.push_back(record(g, r));
        ks.push_back(g.counts[size_t(r)]);
        outs.push_back(g.ids[size_t(r)].data());
      }
      B_.record_ids_batch(recs, ks, ld_, outs);  // one host round trip for all sources
    }
    return g;
  }
  const double* record(const Gathered& g, int r) const { return recv_.as<double>() + int64_t(r) * g.kmax * w_; }

  // Tree: count, then one packed buffer (M3 :689-716).
  void send_set(const DSet& S, int peer) {
    Range tr(B_, "cascade:send_svs");
    auto tm = timer(kPhSendRecv);
    t_.send_i64(S.k, peer);
    if (!S.k) return;
    pack_.ensure(S.k * w_ * 8);
    B_.pack(S, ld_, pack_.as<double>());
    t_.send(pack_.get(), S.k * w_ * 8, peer);
  }
  DSet recv_set(int peer) {
    Range tr(B_, "cascade:recv_svs");
    auto tm = timer(kPhSendRecv);
    const int64_t k = t_.recv_i64(peer);
    pack_.ensure(std::max<int64_t>(k, 1) * w_ * 8);
    if (k) t_.recv(pack_.get(), k * w_ * 8, peer);
    std::vector<int64_t> ids(static_cast<size_t>(k));
    if (k) B_.record_ids(pack_.as<double>(), k, ld_, ids.data());
    Segment s;
    s.rec = pack_.as<double>();
    s.rec_rows = k;
    s.rec_ids = ids.data();
    return assemble({s});
  }

  // ---- checkpoint (rank 0): records of d + 3 doubles, independent of the backend's row stride
  void save_checkpoint(const std::string& dir, bool tree, int64_t next_round, double b, const DSet& G) {
    auto tm = timer(kPhCheckpoint);
    std::vector<double> recs(size_t(G.k) * size_t(d_ + 3));
    if (G.k) {
      pack_.ensure(G.k * w_ * 8);
      B_.pack(G, ld_, pack_.as<double>());
      std::vector<double> wide(size_t(G.k) * size_t(w_));
      B_.d2h(wide.data(), pack_.get(), G.k * w_ * 8);
      for (int64_t i = 0; i < G.k; ++i) {
        std::memcpy(&recs[size_t(i * (d_ + 3))], &wide[size_t(i * w_)], size_t(d_) * 8);
        std::memcpy(&recs[size_t(i * (d_ + 3) + d_)], &wide[size_t(i * w_ + ld_)], 24);
      }
    }
    std::filesystem::create_directories(dir);
    const std::string path = dir + "/cascade_state.bin", tmp = path + ".tmp";
    {
      std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
      if (!f) throw CascadeError("cannot write checkpoint " + tmp);
      const int32_t topo = tree ? 1 : 0, reserved = 0;
      const int64_t d = d_, k = G.k;
      f.write(kCheckpointMagic, 8);
      f.write(reinterpret_cast<const char*>(&topo), 4);
      f.write(reinterpret_cast<const char*>(&reserved), 4);
      f.write(reinterpret_cast<const char*>(&next_round), 8);
      f.write(reinterpret_cast<const char*>(&b), 8);
      f.write(reinterpret_cast<const char*>(&d), 8);
      f.write(reinterpret_cast<const char*>(&k), 8);
      f.write(reinterpret_cast<const char*>(&fingerprint), 8);
      f.write(reinterpret_cast<const char*>(recs.data()), std::streamsize(recs.size() * 8));
      if (!f) throw CascadeError("short write on checkpoint " + tmp);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw CascadeError("cannot rename " + tmp);
  }
  // Returns false when there is no checkpoint file; throws when it does not match this run.
  bool load_checkpoint(const std::string& dir, bool tree, int64_t* next_round, double* b, DSet* G) {
    std::ifstream f(dir + "/cascade_state.bin", std::ios::binary);
    if (!f) return false;
    char magic[8];
    int32_t topo = 0, reserved = 0;
    int64_t d = 0, k = 0;
    uint64_t fp = 0;
    f.read(magic, 8);
    f.read(reinterpret_cast<char*>(&topo), 4);
    f.read(reinterpret_cast<char*>(&reserved), 4);
    f.read(reinterpret_cast<char*>(next_round), 8);
    f.read(reinterpret_cast<char*>(b), 8);
    f.read(reinterpret_cast<char*>(&d), 8);
    f.read(reinterpret_cast<char*>(&k), 8);
    f.read(reinterpret_cast<char*>(&fp), 8);
    if (!f || std::memcmp(magic, kCheckpointMagic, 8) != 0) throw CascadeError("not a cascade checkpoint");
    if (topo != (tree ? 1 : 0) || d != d_ || k < 0 || *next_round < 0)
      throw CascadeError("checkpoint does not match this cascade configuration");
    if (fp != fingerprint)
      throw CascadeError("checkpoint belongs to another training set (row count or column ranges differ)");
    std::vector<double> recs(size_t(k) * size_t(d_ + 3));
    f.read(reinterpret_cast<char*>(recs.data()), std::streamsize(recs.size() * 8));
    if (!f) throw CascadeError("truncated cascade checkpoint");
    std::vector<double> wide(size_t(k) * size_t(w_), 0.0);
    std::vector<int64_t> ids(static_cast<size_t>(k));
    for (int64_t i = 0; i < k; ++i) {
      std::memcpy(&wide[size_t(i * w_)], &recs[size_t(i * (d_ + 3))], size_t(d_) * 8);
      std::memcpy(&wide[size_t(i * w_ + ld_)], &recs[size_t(i * (d_ + 3) + d_)], 24);
      ids[size_t(i)] = int64_t(recs[size_t(i * (d_ + 3) + d_ + 2)]);
    }
    pack_.ensure(std::max<int64_t>(k, 1) * w_ * 8);
    if (k) B_.h2d(pack_.get(), wide.data(), k * w_ * 8);
    Segment s;
    s.rec = pack_.as<double>();
    s.rec_rows = k;
    s.rec_ids = ids.data();
    *G = assemble({s});
    return true;
  }

 private:
  Transport& t_;
  Backend& B_;
  int64_t d_, ld_, w_;
  const CascadeConfig& cfg_;
  Buf pack_, recv_;
  bool prof_ = false;
};

bool same_ids(const DSet& S, const std::unordered_set<int64_t>& prev) {
  if (size_t(S.k) != prev.size()) return false;
  for (int64_t id : S.ids)
    if (!prev.count(id)) return false;
  return true;
}

}  // namespace

CascadeOutput run_cascade(Transport& t, Backend& B, const void* X, bool u8, const int32_t* y, const int64_t* ids,
                          int64_t n_part, int64_t d, int64_t n_total, const CascadeConfig& cfg) {
  const int P = t.world(), me = t.rank();
  const bool log = cfg.log && me == 0;
  const auto t_entry = Clock::now();
  if (cfg.tree && (P & (P - 1)))  // mpi_svm_main3.cpp:420-428 aborts on a non-power-of-2 world
    throw CascadeError("classical (tree) cascade needs a power-of-2 number of ranks, got " + std::to_string(P));
  const int64_t d0 = t.bcast_i64(d, 0);
  if (d0 != d) throw CascadeError("partition feature count differs from rank 0's");
  n_total = t.bcast_i64(n_total, 0);
  if (n_total <= 0) throw CascadeError("No data read from file.");  // MPI_Abort on empty data, M3 :450-454
  Rank R(t, B, d, cfg);
  if (log) {
    printf("[rank 0] Running %s with %d processes\n", cfg.tree ? "CascadeSVM" : "modified CascadeSVM", P);
    printf("[rank 0] total samples = %lld, features = %lld\n", (long long)n_total, (long long)d);
    fflush(stdout);
  }
  const auto t_bc = Clock::now();
  DSet part = R.upload(X, u8, y, ids, n_part);  // data distribution (not timed, M3 :526)
  const auto t_up = Clock::now();
  B.sync();
  const auto t_sy = Clock::now();
  t.barrier();
  if (const char* e = getenv("SVM355_CASCADE_PROFILE"); e && atoi(e) >= 2)
    fprintf(stderr, "[cascade rank %d] setup: bcasts %.3f ms, upload %.3f ms, sync %.3f ms, barrier %.3f ms\n", me,
            ms_between(t_entry, t_bc), ms_between(t_bc, t_up), ms_between(t_up, t_sy), ms_between(t_sy, Clock::now()));

  CascadeOutput out;
  const auto t0 = Clock::now();
  R.phase[kPhSetup] = ms_between(t_entry, t0) - R.phase[kPhUpload];
  R.scale_global(part);
  // with checkpoints, this rank's rows as passed, labels and ids hashed (64-bit words, FNV-1a style; ~10
  // GB/s on the host) and the hashes gathered in rank order
  uint64_t rows_hash = 0;
  if (t.bcast_i64(cfg.checkpoint_dir.empty() ? 0 : 1, 0)) {
    auto hash_words = [](uint64_t h, const void* p, size_t bytes) {
      const auto* c = static_cast<const unsigned char*>(p);
      size_t i = 0;
      for (; i + 8 <= bytes; i += 8) {
        uint64_t w;
        std::memcpy(&w, c + i, 8);
        h = (h ^ w) * 1099511628211ull;
      }
      for (; i < bytes; ++i) h = (h ^ c[i]) * 1099511628211ull;
      return h;
    };
    uint64_t local = 1469598103934665603ull;
    local = hash_words(local, X, size_t(n_part) * size_t(d) * (u8 ? 1 : 8));
    local = hash_words(local, y, size_t(n_part) * 4);
    if (ids) local = hash_words(local, ids, size_t(n_part) * 8);
    for (int64_t v : t.allgather_i64(int64_t(local))) rows_hash = hash_words(rows_hash ^ 0x9E3779B97F4A7C15ull, &v, 8);
  }
  R.fingerprint = R.data_fingerprint(n_total, rows_hash);
  DSet G = R.make(0);  // global SV set (meaningful on rank 0; broadcast each round)
  std::unordered_set<int64_t> global_ids;
  double b = 0.0;
  int rnd = 0;
  if (cfg.resume && !cfg.checkpoint_dir.empty()) {
    int64_t has = 0, next = 0;
    if (me == 0) has = R.load_checkpoint(cfg.checkpoint_dir, cfg.tree, &next, &b, &G) ? 1 : 0;
    if (t.bcast_i64(has, 0)) {
      rnd = int(t.bcast_i64(next, 0));
      global_ids = std::unordered_set<int64_t>(G.ids.begin(), G.ids.end());
      if (log) printf("[rank 0] resumed from checkpoint at round %d, SV count = %lld\n", rnd, (long long)G.k);
    }
  }
  auto tr_prev = Clock::now();
  bool converged = false;
  while (rnd < cfg.max_rounds && !converged) {
    const int shown = cfg.tree ? rnd + 1 : rnd;  // M3 prints rounds from 1 (:571), M2 from 0 (:441)
    Range round_range(B, "cascade:round" + std::to_string(shown));
    if (me == cfg.fail_rank && rnd == cfg.fail_round) {
      if (cfg.fail_stall_s <= 0) throw CascadeError("injected failure at round " + std::to_string(rnd));
      std::this_thread::sleep_for(std::chrono::duration<double>(cfg.fail_stall_s));  // then carries on
    }
    if (log) {
      printf("=== Round %d ===\n", shown);
      fflush(stdout);
    }
    DSet Gb = R.bcast_set(G);
    int64_t same = 0;
    if (!cfg.tree) {
      DSet S = R.merge_unseen(Gb, part);
      DSet local = R.solve(S, shown, 0, Gb.k, true).first;
      const auto g = R.gather_sets(local);
      if (me == 0) {
        // merged = own SVs (alphas kept) U unseen worker SVs in source order 1..P-1 with their
        // alphas reset to 0 (M2 :552-607, :600-601)
        std::unordered_set<int64_t> seen(local.ids.begin(), local.ids.end());
        std::vector<std::vector<int64_t>> keep(static_cast<size_t>(P));
        std::vector<Segment> segs{Segment{&local, nullptr, 0, nullptr, nullptr, false}};
        for (int src = 1; src < P; ++src) {
          const int64_t c = g.counts[size_t(src)];
          for (int64_t i = 0; i < c; ++i) {
            const int64_t id = g.ids[size_t(src)][size_t(i)];
            if (seen.insert(id).second) keep[size_t(src)].push_back(i);
          }
          Segment s;
          s.rec = R.record(g, src);
          s.rec_rows = c;
          s.rec_ids = g.ids[size_t(src)].data();
          s.idx = &keep[size_t(src)];
          s.zero_alpha = true;
          segs.push_back(s);
        }
        DSet merged = [&] {
          auto tm = R.timer(kPhAssemble);
          return R.assemble(segs);
        }();
        out.merged_history.push_back(merged.k);
        if (log) printf("[rank 0] merged unique SV count from workers = %lld\n", (long long)merged.k);
        auto res = R.solve(merged, shown, -1);
        b = res.second;
        same = same_ids(res.first, global_ids);
        G = std::move(res.first);
        global_ids = std::unordered_set<int64_t>(G.ids.begin(), G.ids.end());
        const auto tr = Clock::now();
        out.round_ms.push_back(ms_between(tr_prev, tr));
        if (log) printf("[rank 0] Round%d takes %d ms\n", shown, int(ms_between(tr_prev, tr)));
        tr_prev = tr;
      }
    } else {
      DSet own = R.make(0);
      const DSet* cur = &part;
      DSet recv = std::move(Gb);
      for (int step = 1; step <= P; step *= 2) {
        if (me % step == 0) {  // receiver's SVs warm, own rows not among them cold (M3 :629-660)
          DSet S = R.merge_unseen(recv, *cur);
          auto res = R.solve(S, shown, step, recv.k, !(me == 0 && step == P));
          own = std::move(res.first);
          cur = &own;
          if (me == 0) b = res.second;
        }
        if (step < P) {
          if (me % (2 * step) == step)
            R.send_set(*cur, me - step);
          else if (me % (2 * step) == 0)
            recv = R.recv_set(me + step);
        }
      }
      if (me == 0) {  // rank 0 solves at every layer, so `own` is its final-layer set
        same = same_ids(own, global_ids);
        G = std::move(own);
        global_ids = std::unordered_set<int64_t>(G.ids.begin(), G.ids.end());
        const auto tr = Clock::now();
        out.round_ms.push_back(ms_between(tr_prev, tr));
        tr_prev = tr;
      }
    }
    if (me == 0) {
      out.sv_history.push_back(G.k);
      if (log) {
        if (same)
          printf("[rank 0] Converged at round %d, SV count = %lld\n", shown, (long long)G.k);
        else
          printf("[rank 0] Not converged yet. New SV count = %lld\n", (long long)G.k);
        fflush(stdout);
      }
      if (!cfg.checkpoint_dir.empty()) R.save_checkpoint(cfg.checkpoint_dir, cfg.tree, rnd + 1, b, G);
    }
    converged = t.bcast_i64(same, 0) != 0;
    ++rnd;
  }
  // Share the final model with every rank (the reference keeps it on rank 0 only).
  const auto t_final = Clock::now();
  const double bcast_before = R.phase[kPhBcast];  // the final broadcast is charged to kPhFinal
  int64_t bbits = 0;
  std::memcpy(&bbits, &b, 8);
  bbits = t.bcast_i64(bbits, 0);
  std::memcpy(&b, &bbits, 8);
  DSet F = R.bcast_set(G);
  B.sync();
  out.train_ms = ms_between(t0, Clock::now());
  out.b = b;
  out.rounds = rnd;
  out.converged = converged;
  out.ids = F.ids;
  out.y.resize(size_t(F.k));
  out.alpha.resize(size_t(F.k));
  if (F.k) {
    B.d2h(out.y.data(), F.y.get(), F.k * 4);
    B.d2h(out.alpha.data(), F.a.get(), F.k * 8);
  }
  out.d = d;
  out.ld = B.ld(d);
  out.final_set = std::move(F);
  out.mn = R.mn_h;
  out.mx = R.mx_h;
  out.solves = std::move(R.log);
  R.phase[kPhBcast] = bcast_before;
  R.phase[kPhFinal] += ms_between(t_final, Clock::now());
  std::copy(R.phase, R.phase + kNumPhases, out.phase_ms);
  if (log) {
    printf("[rank 0] Final b = %.15f\n", b);
    fflush(stdout);
  }
  return out;
}

}  // namespace svm355
