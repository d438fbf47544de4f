// Native Cascade SVM driver (see cascade.h).  Rows stay on the rank's device end to end: an SV set
// is device rows (k x ld) plus host labels / alphas / ids, and travels as ONE packed device buffer
// of k x (ld + 3) doubles [row | y | alpha | id] (ids < 2^53 and +-1 labels are exact in float64),
// so each exchange is a count plus one bulk transfer.
#include "cascade.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <numeric>
#include <stdexcept>
#include <unordered_set>
#include <utility>

#include "svm355_device.h"

namespace svm355 {
namespace {

#define SVMC(expr)                                                                                  \
  do {                                                                                              \
    if ((expr) != SVM_OK) throw std::runtime_error(std::string(#expr) + ": " + svm_last_error());   \
  } while (0)
#define HIPC(expr)                                                                                  \
  do {                                                                                              \
    const hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// roctx range through the device library (visible with rocprofv3 --marker-trace), SURVEY §5.1.
struct Trace {
  explicit Trace(const std::string& name) { svmd_trace_push(name.c_str()); }
  ~Trace() { svmd_trace_pop(); }
  Trace(const Trace&) = delete;
  Trace& operator=(const Trace&) = delete;
};

using Clock = std::chrono::steady_clock;
double ms_between(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

// Grow-only device buffer from the svmd context allocator.
struct DevBuf {
  void* ctx = nullptr;
  void* p = nullptr;
  int64_t bytes = 0;
  explicit DevBuf(void* c = nullptr) : ctx(c) {}
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : ctx(o.ctx), p(o.p), bytes(o.bytes) {
    o.p = nullptr;
    o.bytes = 0;
  }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      reset();
      ctx = o.ctx;
      p = o.p;
      bytes = o.bytes;
      o.p = nullptr;
      o.bytes = 0;
    }
    return *this;
  }
  ~DevBuf() { reset(); }
  void reset() {
    if (p) svmd_free(ctx, p);
    p = nullptr;
    bytes = 0;
  }
  void ensure(int64_t b) {  // contents are not preserved when it grows
    if (b <= bytes) return;
    reset();
    p = svmd_alloc(ctx, std::max<int64_t>(b, 8));
    if (!p) throw std::runtime_error(std::string("svmd_alloc: ") + svm_last_error());
    bytes = b;
  }
  void* release() {
    void* q = p;
    p = nullptr;
    bytes = 0;
    return q;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct SvSet {
  DevBuf X;  // k x ld rows
  int64_t k = 0;
  std::vector<int32_t> y;
  std::vector<double> alpha;
  std::vector<int64_t> ids;
};

class Rank {
 public:
  Rank(Transport& t, void* ctx, int64_t d, const CascadeConfig& cfg)
      : t_(t), ctx_(ctx), d_(d), ld_(svmd_padded_dim(d)), w_(ld_ + 3), cfg_(cfg), K_(ctx), sqn_(ctx), yd_(ctx),
        ad_(ctx), idx_(ctx), pack_(ctx), recvbuf_(ctx), cnt_(ctx) {
    HIPC(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  }
  ~Rank() { (void)hipStreamDestroy(stream_); }

  int64_t ld() const { return ld_; }
  int64_t solves = 0, iterations = 0;
  std::vector<double> mn_h, mx_h;

  SvSet empty() {
    SvSet s;
    s.X = DevBuf(ctx_);
    return s;
  }
  void sync() { SVMC(svmd_synchronize(ctx_)); }

  // Upload and scale this rank's partition with the globally all-reduced column min / max
  // (bitwise equal to the reference's rank-0 min/max + MPI_Bcast, M3 :529-539).
  SvSet upload(const double* X, const int32_t* y, const int64_t* ids, int64_t n) {
    SvSet s = empty();
    s.k = n;
    s.X.ensure(n * ld_ * 8);
    if (n) SVMC(svmd_upload_rows(ctx_, X, n, d_, s.X.as<double>(), ld_));
    s.y.assign(y, y + n);
    s.alpha.assign(size_t(n), 0.0);
    s.ids.assign(ids, ids + n);
    sync();
    return s;
  }
  void scale_global(SvSet& part) {
    DevBuf mn(ctx_), mx(ctx_);
    mn.ensure(d_ * 8);
    mx.ensure(d_ * 8);
    if (part.k) {
      SVMC(svmd_minmax(ctx_, part.X.as<double>(), part.k, d_, ld_, mn.as<double>(), mx.as<double>()));
    } else {  // an empty partition contributes the identities of min / max
      std::vector<double> hi(size_t(d_), __builtin_inf()), lo(size_t(d_), -__builtin_inf());
      SVMC(svmd_memcpy_h2d(ctx_, mn.p, hi.data(), d_ * 8));
      SVMC(svmd_memcpy_h2d(ctx_, mx.p, lo.data(), d_ * 8));
    }
    sync();
    t_.allreduce_min(mn.as<double>(), d_);
    t_.allreduce_max(mx.as<double>(), d_);
    if (part.k) {
      DevBuf nrm(ctx_);
      nrm.ensure(part.k * 8);
      SVMC(svmd_preprocess(ctx_, part.X.as<double>(), part.k, d_, ld_, mn.as<double>(), mx.as<double>(),
                           nrm.as<double>(), 1));
    }
    mn_h.resize(size_t(d_));
    mx_h.resize(size_t(d_));
    SVMC(svmd_memcpy_d2h(ctx_, mn_h.data(), mn.p, d_ * 8));
    SVMC(svmd_memcpy_d2h(ctx_, mx_h.data(), mx.p, d_ * 8));
  }

  // Rows `keep` of S (ascending as given), alphas zeroed on request.
  SvSet subset(const SvSet& S, const std::vector<int64_t>& keep, bool zero_alpha) {
    SvSet o = empty();
    o.k = int64_t(keep.size());
    o.X.ensure(o.k * ld_ * 8);
    if (o.k) {
      idx_.ensure(o.k * 8);
      SVMC(svmd_memcpy_h2d(ctx_, idx_.p, keep.data(), o.k * 8));
      SVMC(svmd_gather_rows(ctx_, S.X.as<double>(), ld_, idx_.as<int64_t>(), o.k, o.X.as<double>()));
      sync();
    }
    o.y.reserve(keep.size());
    o.alpha.reserve(keep.size());
    o.ids.reserve(keep.size());
    for (int64_t i : keep) {
      o.y.push_back(S.y[size_t(i)]);
      o.alpha.push_back(zero_alpha ? 0.0 : S.alpha[size_t(i)]);
      o.ids.push_back(S.ids[size_t(i)]);
    }
    return o;
  }
  SvSet concat(const SvSet& a, const SvSet& b) {
    SvSet o = empty();
    o.k = a.k + b.k;
    o.X.ensure(o.k * ld_ * 8);
    sync();
    if (a.k) HIPC(hipMemcpyAsync(o.X.p, a.X.p, size_t(a.k * ld_ * 8), hipMemcpyDeviceToDevice, stream_));
    if (b.k)
      HIPC(hipMemcpyAsync(o.X.as<double>() + a.k * ld_, b.X.p, size_t(b.k * ld_ * 8), hipMemcpyDeviceToDevice,
                          stream_));
    HIPC(hipStreamSynchronize(stream_));
    for (const SvSet* s : {&a, &b}) {
      o.y.insert(o.y.end(), s->y.begin(), s->y.end());
      o.alpha.insert(o.alpha.end(), s->alpha.begin(), s->alpha.end());
      o.ids.insert(o.ids.end(), s->ids.begin(), s->ids.end());
    }
    return o;
  }
  // warm (alphas kept) U rows of extra whose id is not in warm (alpha = 0), extra order kept
  // (the seen_ids loops of mpi_svm_main3.cpp:629-655 / mpi_svm_main2.cpp:474-502).
  SvSet merge_unseen(const SvSet& warm, const SvSet& extra) {
    std::vector<int64_t> keep;
    keep.reserve(size_t(extra.k));
    if (warm.k == 0) {
      keep.resize(size_t(extra.k));
      std::iota(keep.begin(), keep.end(), int64_t(0));
      return subset(extra, keep, true);
    }
    const std::unordered_set<int64_t> seen(warm.ids.begin(), warm.ids.end());
    for (int64_t i = 0; i < extra.k; ++i)
      if (!seen.count(extra.ids[size_t(i)])) keep.push_back(i);
    return concat(warm, subset(extra, keep, true));
  }

  // ---- packing: k x (ld + 3) doubles [row | y | alpha | id]
  void pack_into(const SvSet& S, DevBuf& buf, int64_t rows_capacity) {
    buf.ensure(std::max<int64_t>(rows_capacity, 1) * w_ * 8);
    if (!S.k) return;
    sync();
    HIPC(hipMemcpy2DAsync(buf.p, size_t(w_ * 8), S.X.p, size_t(ld_ * 8), size_t(ld_ * 8), size_t(S.k),
                          hipMemcpyDeviceToDevice, stream_));
    std::vector<double> tail(size_t(S.k) * 3);
    for (int64_t i = 0; i < S.k; ++i) {
      tail[size_t(3 * i)] = double(S.y[size_t(i)]);
      tail[size_t(3 * i + 1)] = S.alpha[size_t(i)];
      tail[size_t(3 * i + 2)] = double(S.ids[size_t(i)]);
    }
    HIPC(hipMemcpy2DAsync(buf.as<double>() + ld_, size_t(w_ * 8), tail.data(), 24, 24, size_t(S.k),
                          hipMemcpyHostToDevice, stream_));
    HIPC(hipStreamSynchronize(stream_));
  }
  SvSet unpack(const double* buf_d, int64_t k) {
    SvSet o = empty();
    o.k = k;
    o.X.ensure(k * ld_ * 8);
    if (!k) return o;
    std::vector<double> tail(size_t(k) * 3);
    HIPC(hipMemcpy2DAsync(o.X.p, size_t(ld_ * 8), buf_d, size_t(w_ * 8), size_t(ld_ * 8), size_t(k),
                          hipMemcpyDeviceToDevice, stream_));
    HIPC(hipMemcpy2DAsync(tail.data(), 24, buf_d + ld_, size_t(w_ * 8), 24, size_t(k), hipMemcpyDeviceToHost,
                          stream_));
    HIPC(hipStreamSynchronize(stream_));
    o.y.resize(size_t(k));
    o.alpha.resize(size_t(k));
    o.ids.resize(size_t(k));
    for (int64_t i = 0; i < k; ++i) {
      o.y[size_t(i)] = int32_t(tail[size_t(3 * i)]);
      o.alpha[size_t(i)] = tail[size_t(3 * i + 1)];
      o.ids[size_t(i)] = int64_t(tail[size_t(3 * i + 2)]);
    }
    return o;
  }

  // ---- checkpoint (rank 0): packed records through the host
  std::vector<double> pack_host(const SvSet& S) {
    std::vector<double> h(size_t(S.k) * size_t(w_));
    if (!S.k) return h;
    pack_into(S, pack_, S.k);
    HIPC(hipMemcpyAsync(h.data(), pack_.p, h.size() * 8, hipMemcpyDeviceToHost, stream_));
    HIPC(hipStreamSynchronize(stream_));
    return h;
  }
  SvSet unpack_host(const std::vector<double>& h, int64_t k) {
    pack_.ensure(std::max<int64_t>(k, 1) * w_ * 8);
    if (k) {
      sync();
      HIPC(hipMemcpyAsync(pack_.p, h.data(), size_t(k) * size_t(w_) * 8, hipMemcpyHostToDevice, stream_));
      HIPC(hipStreamSynchronize(stream_));
    }
    return unpack(pack_.as<double>(), k);
  }
  void save_checkpoint(const std::string& dir, bool tree, int64_t next_round, double b, const SvSet& G) {
    const std::vector<double> recs = pack_host(G);
    std::filesystem::create_directories(dir);
    const std::string path = dir + "/cascade_state.bin", tmp = path + ".tmp";
    {
      std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
      if (!f) throw std::runtime_error("cannot write checkpoint " + tmp);
      const int32_t topo = tree ? 1 : 0, reserved = 0;
      const int64_t d = d_, ld = ld_, k = G.k;
      f.write(kCheckpointMagic, 8);
      f.write(reinterpret_cast<const char*>(&topo), 4);
      f.write(reinterpret_cast<const char*>(&reserved), 4);
      f.write(reinterpret_cast<const char*>(&next_round), 8);
      f.write(reinterpret_cast<const char*>(&b), 8);
      f.write(reinterpret_cast<const char*>(&d), 8);
      f.write(reinterpret_cast<const char*>(&ld), 8);
      f.write(reinterpret_cast<const char*>(&k), 8);
      f.write(reinterpret_cast<const char*>(recs.data()), std::streamsize(recs.size() * 8));
      if (!f) throw std::runtime_error("short write on checkpoint " + tmp);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("cannot rename " + tmp);
  }
  // Returns false when there is no checkpoint file; throws when it does not match this run.
  bool load_checkpoint(const std::string& dir, bool tree, int64_t* next_round, double* b, SvSet* G) {
    std::ifstream f(dir + "/cascade_state.bin", std::ios::binary);
    if (!f) return false;
    char magic[8];
    int32_t topo = 0, reserved = 0;
    int64_t d = 0, ld = 0, k = 0;
    f.read(magic, 8);
    f.read(reinterpret_cast<char*>(&topo), 4);
    f.read(reinterpret_cast<char*>(&reserved), 4);
    f.read(reinterpret_cast<char*>(next_round), 8);
    f.read(reinterpret_cast<char*>(b), 8);
    f.read(reinterpret_cast<char*>(&d), 8);
    f.read(reinterpret_cast<char*>(&ld), 8);
    f.read(reinterpret_cast<char*>(&k), 8);
    if (!f || std::memcmp(magic, kCheckpointMagic, 8) != 0) throw std::runtime_error("not a cascade checkpoint");
    if (topo != (tree ? 1 : 0) || d != d_ || ld != ld_ || k < 0)
      throw std::runtime_error("checkpoint does not match this cascade configuration");
    std::vector<double> recs(size_t(k) * size_t(w_));
    f.read(reinterpret_cast<char*>(recs.data()), std::streamsize(recs.size() * 8));
    if (!f) throw std::runtime_error("truncated cascade checkpoint");
    *G = unpack_host(recs, k);
    return true;
  }

  // ---- exchanges
  SvSet bcast_set(const SvSet& G) {  // G meaningful on rank 0
    Trace tr("cascade:bcast_svs");
    const int64_t k = t_.bcast_i64(t_.rank() == 0 ? G.k : 0, 0);
    if (t_.rank() == 0)
      pack_into(G, pack_, k);
    else
      pack_.ensure(std::max<int64_t>(k, 1) * w_ * 8);
    t_.bcast(pack_.p, k * w_ * 8, 0);
    return unpack(pack_.as<double>(), k);
  }
  // Star: local SV sets to rank 0 (counts all-gathered, max-count-padded gather, source order).
  std::vector<SvSet> gather_sets(const SvSet& local) {
    Trace tr("cascade:gather_svs");
    const std::vector<int64_t> counts = t_.allgather_i64(local.k);
    const int64_t kmax = *std::max_element(counts.begin(), counts.end());
    std::vector<SvSet> out;
    if (kmax == 0) {
      if (t_.rank() == 0)
        for (size_t r = 0; r < counts.size(); ++r) out.push_back(empty());
      return out;
    }
    pack_into(local, pack_, kmax);
    const int64_t bytes = kmax * w_ * 8;
    if (t_.rank() == 0) recvbuf_.ensure(bytes * t_.world());
    t_.gather(pack_.p, bytes, t_.rank() == 0 ? recvbuf_.p : nullptr, 0);
    if (t_.rank() == 0)
      for (int r = 0; r < t_.world(); ++r)
        out.push_back(unpack(recvbuf_.as<double>() + int64_t(r) * kmax * w_, counts[size_t(r)]));
    return out;
  }
  // Tree: count, then one packed buffer (M3 :689-716).
  void send_set(const SvSet& S, int peer) {
    Trace tr("cascade:send_svs");
    cnt_.ensure(8);
    SVMC(svmd_memcpy_h2d(ctx_, cnt_.p, &S.k, 8));
    t_.send(cnt_.p, 8, peer);
    if (S.k) {
      pack_into(S, pack_, S.k);
      t_.send(pack_.p, S.k * w_ * 8, peer);
    }
  }
  SvSet recv_set(int peer) {
    Trace tr("cascade:recv_svs");
    cnt_.ensure(8);
    t_.recv(cnt_.p, 8, peer);
    int64_t k = 0;
    SVMC(svmd_memcpy_d2h(ctx_, &k, cnt_.p, 8));
    pack_.ensure(std::max<int64_t>(k, 1) * w_ * 8);
    if (k) t_.recv(pack_.p, k * w_ * 8, peer);
    return unpack(pack_.as<double>(), k);
  }

  // Warm-start SMO on S (SMO_train(..., init=false)); returns (its SVs with alpha > sv_tol, b).
  std::pair<SvSet, double> solve(const SvSet& S) {
    if (S.k == 0) return {empty(), 0.0};
    Trace tr("cascade:solve");
    const int64_t k = S.k, ldk = (k + 1) / 2 * 2;
    sqn_.ensure(k * 8);
    yd_.ensure(k * 4);
    ad_.ensure(k * 8);
    K_.ensure(k * ldk * 8);
    SVMC(svmd_row_norms(ctx_, S.X.as<double>(), k, d_, ld_, sqn_.as<double>()));
    SVMC(svmd_memcpy_h2d(ctx_, yd_.p, S.y.data(), k * 4));
    SVMC(svmd_memcpy_h2d(ctx_, ad_.p, S.alpha.data(), k * 8));
    svm_result r{};
    svmd_timing tm{};
    int32_t used = 0;
    SVMC(svmd_train_q(ctx_, S.X.as<double>(), sqn_.as<double>(), k, ld_, ld_, yd_.as<int32_t>(), ad_.as<double>(), 1,
                      &cfg_.params, &r, K_.as<double>(), ldk, &tm, mn_h.data(), mx_h.data(), d_, 0, &used));
    std::vector<double> a(static_cast<size_t>(k));
    SVMC(svmd_memcpy_d2h(ctx_, a.data(), ad_.p, k * 8));
    ++solves;
    iterations += r.iterations;
    std::vector<int64_t> keep;
    for (int64_t i = 0; i < k; ++i)
      if (a[size_t(i)] > cfg_.params.sv_tol) keep.push_back(i);
    SvSet out = subset(S, keep, false);
    for (size_t j = 0; j < keep.size(); ++j) out.alpha[j] = a[size_t(keep[j])];
    return {std::move(out), r.b};
  }

 private:
  Transport& t_;
  void* ctx_;
  int64_t d_, ld_, w_;
  CascadeConfig cfg_;
  DevBuf K_, sqn_, yd_, ad_, idx_, pack_, recvbuf_, cnt_;
  hipStream_t stream_ = nullptr;
};

bool same_ids(const SvSet& S, const std::unordered_set<int64_t>& prev) {
  if (size_t(S.k) != prev.size()) return false;
  for (int64_t id : S.ids)
    if (!prev.count(id)) return false;
  return true;
}

}  // namespace

CascadeOutput run_cascade(Transport& t, void* ctx, const double* X_host, const int32_t* y_host,
                          const int64_t* ids_host, int64_t n_part, int64_t d, int64_t n_total,
                          const CascadeConfig& cfg) {
  const int P = t.world(), me = t.rank();
  const bool log = cfg.log && me == 0;
  if (cfg.tree && (P & (P - 1)))  // mpi_svm_main3.cpp:420-428 aborts on a non-power-of-2 world
    throw std::runtime_error("classical (tree) cascade needs a power-of-2 number of ranks");
  const int64_t d0 = t.bcast_i64(d, 0);
  if (d0 != d) throw std::runtime_error("partition feature count differs from rank 0's");
  n_total = t.bcast_i64(n_total, 0);
  Rank R(t, ctx, d, cfg);
  if (log) {
    printf("[rank 0] Running %s with %d processes\n", cfg.tree ? "CascadeSVM" : "modified CascadeSVM", P);
    printf("[rank 0] total samples = %lld, features = %lld\n", (long long)n_total, (long long)d);
    fflush(stdout);
  }
  SvSet part = R.upload(X_host, y_host, ids_host, n_part);  // data distribution (not timed, M3 :526)
  t.barrier();

  CascadeOutput out;
  const auto t0 = Clock::now();
  R.scale_global(part);
  SvSet G = R.empty();  // global SV set (meaningful on rank 0; broadcast each round)
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
    const int shown = cfg.tree ? rnd + 1 : rnd;
    Trace round_range("cascade:round" + std::to_string(shown));
    if (log) {
      printf("=== Round %d ===\n", shown);
      fflush(stdout);
    }
    SvSet Gb = R.bcast_set(G);
    int64_t same = 0;
    if (!cfg.tree) {
      auto local = R.solve(R.merge_unseen(Gb, part)).first;
      std::vector<SvSet> got = R.gather_sets(local);
      if (me == 0) {
        SvSet merged = std::move(local);
        std::unordered_set<int64_t> seen(merged.ids.begin(), merged.ids.end());
        for (int src = 1; src < P; ++src) {  // source order 1..P-1 (M2 :578); worker alphas reset (:600-601)
          const SvSet& w = got[size_t(src)];
          std::vector<int64_t> keep;
          for (int64_t i = 0; i < w.k; ++i)
            if (!seen.count(w.ids[size_t(i)])) keep.push_back(i);
          for (int64_t i : keep) seen.insert(w.ids[size_t(i)]);
          merged = R.concat(merged, R.subset(w, keep, true));
        }
        out.merged_history.push_back(merged.k);
        if (log) printf("[rank 0] merged unique SV count from workers = %lld\n", (long long)merged.k);
        auto res = R.solve(merged);
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
      const SvSet* cur = &part;
      SvSet cur_own = R.empty();
      SvSet recv = std::move(Gb);
      for (int step = 1; step <= P; step *= 2) {
        if (me % step == 0) {
          auto res = R.solve(R.merge_unseen(recv, *cur));
          cur_own = std::move(res.first);
          cur = &cur_own;
          if (me == 0) b = res.second;
        }
        if (step < P) {
          if (me % (2 * step) == step)
            R.send_set(*cur, me - step);
          else if (me % (2 * step) == 0)
            recv = R.recv_set(me + step);
        }
      }
      if (me == 0) {  // rank 0 solves at every layer, so cur_own is its final-layer set
        same = same_ids(cur_own, global_ids);
        G = std::move(cur_own);
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
  int64_t bbits = 0;
  std::memcpy(&bbits, &b, 8);
  bbits = t.bcast_i64(bbits, 0);
  std::memcpy(&b, &bbits, 8);
  SvSet F = R.bcast_set(G);
  R.sync();
  out.train_ms = ms_between(t0, Clock::now());
  out.b = b;
  out.rounds = rnd;
  out.converged = converged;
  out.ids = F.ids;
  out.y = F.y;
  out.alpha = F.alpha;
  out.X_d = static_cast<double*>(F.X.release());
  out.mn = R.mn_h;
  out.mx = R.mx_h;
  out.solves = R.solves;
  out.iterations = R.iterations;
  if (log) {
    printf("[rank 0] Final b = %.15f\n", b);
    fflush(stdout);
  }
  return out;
}

}  // namespace svm355
