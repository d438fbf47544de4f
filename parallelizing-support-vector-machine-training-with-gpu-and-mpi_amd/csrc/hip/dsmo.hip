// Distributed first-order SMO over the GPUs of one node (opt-in `--parallel smo`).
//
// The reference scales past one processor only with the Cascade SVM (mpi_svm_main2/3.cpp), whose
// rounds re-solve partitions and merged SV sets: at the 60k headline its rank 0 runs ~4x the
// iterations of one SMO (profiles/r2_cascade_critical_path.txt).  Its literature folder holds the
// alternative (papers/2006_Cao_SVM_MPI.pdf): ONE SMO whose O(n) inner loops are split
// over the processors, with a global arg-min / arg-max every iteration.  On MI355X that is the
// persistent solver (persist.h) with its teams spread over GPUs:
//
//   * team t (one per GPU) owns points [t*W, (t+1)*W) and computes its slab K(:, own) of the
//     exact-integer RBF Gram (igram RECT, n x W: 1/P of the Gram's work and memory -- 537k points
//     fit resident in 8 x 288 GB where one GPU falls to the row cache above 189k);
//   * every iteration each workgroup stores its candidate record into the receive array of every
//     team -- its own GPU's and, over xGMI, its peers' (uncached fine-grained memory, system-scope
//     stores of self-validating granules, dsmo.h) -- and sweeps only its own GPU's array, so the
//     exchange costs one fabric hop, not a round trip;
//   * K12 = K(i_high, i_low), which lives in one team's slab, is recomputed by every wave from the
//     two quantised rows with the Gram's exact arithmetic (k12_exact) while the slab reads are in
//     flight, so no second exchange is needed and every workgroup applies the identical update.
// The values are the resident Gram's and the reductions keep the lowest-index rule, so the
// trajectory -- every (i_high, i_low), alpha and b -- is the single-GPU solve's, bit for bit.
//
// Launch forms (one code path):
//   * P GPUs of this process, one host thread and one launch per GPU (peer access enabled between
//     them), or
//   * a rehearsal: P teams in ONE launch on one GPU (uncached receive arrays in its own HBM), which
//     checks the trajectory and measures the exchange through uncached memory without peers.
// Every spin is bounded (a peer that never launches or dies ends every workgroup's wait with an
// error).  Before a timed run, bench.py's preflight solves 4,096 rows distributed and on one GPU and
// requires the same iterations, b and alphas (bench.py, PREFLIGHT_ROWS).
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "cascade.h"
#include "persist.h"
#include "svm355_device.h"
#include "trace.h"

namespace svm355 {
namespace {

struct DsmoArgs {
  DsmoTeam team[kMaxPeers];
  PeerExch px;
  int teams;         // P
  int Gt;            // workgroups per team
  int team_base;     // team of this launch's first workgroup
  uint32_t epoch0;   // record tags continue from here (never reused on the receive arrays)
};

__global__ void dsmo_init_kernel(const int32_t* __restrict__ y, double* __restrict__ alpha, double* __restrict__ f,
                                 int64_t n, SmoState* __restrict__ st, int nst) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) {
    alpha[i] = 0.0;
    f[i] = -static_cast<double>(y[i]);  // cold start, main3.cpp:165-172
  }
  if (i < nst) st[i] = SmoState{0, 0, 0.0, 0.0, 0.0, 0.0, 1, 0, SVM_STOP_RUNNING};
}

// Workgroup b of a launch: team team_base + b / Gt, global workgroup index team * Gt + b % Gt, so the
// slices of all teams tile [0, n) contiguously and team t's points are its slab's columns.
template <int NT, int E, int RPL>
__global__ __launch_bounds__(NT) void smo_dsmo_kernel(DsmoArgs a, QRows q, double neg_gamma,
                                                      const int32_t* __restrict__ y, double* __restrict__ alpha,
                                                      double* __restrict__ f, int64_t n, int64_t slice,
                                                      SmoState* __restrict__ st, double C, double eps, double tau,
                                                      int64_t max_iter, int64_t* __restrict__ trace, int64_t trace_cap,
                                                      unsigned* __restrict__ err, int64_t spin_limit) {
  __shared__ PersistShared sh;
  const int tl = int(blockIdx.x) / a.Gt;
  const int team = a.team_base + tl;
  const int g = team * a.Gt + (int(blockIdx.x) - tl * a.Gt);
  PeerExch px = a.px;
  px.own = team;
  const DsmoTeam tm = a.team[team];
  const SlabRows rows{tm.slab, tm.ldw, tm.col0, q, neg_gamma};
  persist_solve<NT, E, false, false, SlabRows, RPL, false, true>(
      sh, a.teams * a.Gt, g, a.epoch0, rows, y, alpha, f, n, slice, nullptr, st + team, C, eps, tau, max_iter,
      team == 0 ? trace : nullptr, trace_cap, err, spin_limit, nullptr, px, team * a.Gt);
}

constexpr int kRecPerArray = 256;  // records per epoch parity of a receive array (RPL <= 4)
constexpr size_t kUcBytes = size_t(2) * kRecPerArray * kRecStride * 8;
// Bound of one exchange wait in s_memrealtime ticks (100 MHz): 2 s, which also absorbs the launch
// skew between GPUs; a peer that never publishes ends every workgroup's wait with an error.
constexpr int64_t kDsmoSpins = 200000000;

struct Shape {
  int NT = 0, E = 0, Gt = 0, RPL = 0;
  int64_t slice = 0, W = 0;
};

// Smallest register footprint whose team fits one sweep of <= 64 records in total, else 128, else
// 256 (RPL 1 / 2 / 4); wg_dev caps the workgroups co-resident on one GPU (all teams of a rehearsal).
bool dsmo_shape(int64_t n, int P, int wg_dev, bool one_launch, Shape* out) {
  static const int cand[][2] = {{256, 2}, {256, 4}, {256, 8}, {512, 4}, {512, 8}};
  int fNT = 0, fE = 0;
  if (const char* v = getenv("SVM355_DSMO_SHAPE")) sscanf(v, "%d,%d", &fNT, &fE);
  const int64_t per = (n + P - 1) / P;
  for (int cap : {64, 128, 256}) {
    for (const auto& c : cand) {
      if (fNT && (c[0] != fNT || c[1] != fE)) continue;
      const int64_t slice = int64_t(c[0]) * c[1];
      const int64_t Gt = std::max<int64_t>(1, (per + slice - 1) / slice);
      const int64_t total = Gt * P;
      if (total > cap) continue;
      if ((one_launch ? total : Gt) > wg_dev) continue;
      out->NT = c[0];
      out->E = c[1];
      out->Gt = int(Gt);
      out->RPL = cap / 64;
      out->slice = slice;
      out->W = Gt * slice;
      return true;
    }
  }
  return false;
}

// Host-side check of everything the kernel and its grid assume (before any launch).
void check_plan(int64_t n, int P, int ncu, bool one_launch, const Shape& sh) {
  const int64_t total = int64_t(P) * sh.Gt;
  auto bad = [&](const char* what) {
    throw CascadeError(std::string("dsmo plan: ") + what + " (n=" + std::to_string(n) + " P=" + std::to_string(P) +
                       " NT=" + std::to_string(sh.NT) + " E=" + std::to_string(sh.E) + " Gt=" + std::to_string(sh.Gt) +
                       " RPL=" + std::to_string(sh.RPL) + ")");
  };
  if (P < 1 || P > kMaxPeers) bad("team count out of range");
  if (sh.slice != int64_t(sh.NT) * sh.E || sh.W != int64_t(sh.Gt) * sh.slice) bad("inconsistent slice / width");
  if (total > int64_t(64) * sh.RPL || total > kRecPerArray) bad("more records than one sweep / array holds");
  if (total * sh.slice < n) bad("the teams do not cover every point");
  if ((one_launch ? total : int64_t(sh.Gt)) > ncu) bad("workgroups of one launch exceed the CUs (not co-resident)");
  if (n >= int64_t(kSentinel)) bad("n too large for 32-bit indices");
}

template <int NT, int E, int RPL>
void launch_e(hipStream_t s, int grid, const DsmoArgs& a, const QRows& q, double ng, const int32_t* y, double* alpha,
              double* f, int64_t n, int64_t slice, SmoState* st, const svm_params& p, int64_t* trace, int64_t tcap,
              unsigned* err) {
  hipLaunchKernelGGL((smo_dsmo_kernel<NT, E, RPL>), dim3(grid), dim3(NT), 0, s, a, q, ng, y, alpha, f, n, slice, st,
                     p.C, p.eps, p.tau, p.max_iter, trace, tcap, err, kDsmoSpins);
}

int launch_dsmo(hipStream_t s, const Shape& sh, int grid, const DsmoArgs& a, const QRows& q, double ng,
                const int32_t* y, double* alpha, double* f, int64_t n, SmoState* st, const svm_params& p,
                int64_t* trace, int64_t tcap, unsigned* err) {
#define SVM_DSMO_CASE(nt, e, r)                                                                                   \
  if (sh.NT == nt && sh.E == e && sh.RPL == r) {                                                                  \
    launch_e<nt, e, r>(s, grid, a, q, ng, y, alpha, f, n, sh.slice, st, p, trace, tcap, err);                     \
    SVMD_LAUNCH_CHECK();                                                                                          \
    return SVM_OK;                                                                                                \
  }
  SVM_DSMO_CASE(256, 2, 1) SVM_DSMO_CASE(256, 4, 1) SVM_DSMO_CASE(256, 8, 1) SVM_DSMO_CASE(512, 4, 1)
  SVM_DSMO_CASE(512, 8, 1)
  SVM_DSMO_CASE(256, 2, 2) SVM_DSMO_CASE(256, 4, 2) SVM_DSMO_CASE(256, 8, 2) SVM_DSMO_CASE(512, 4, 2)
  SVM_DSMO_CASE(512, 8, 2)
  SVM_DSMO_CASE(256, 2, 4) SVM_DSMO_CASE(256, 4, 4) SVM_DSMO_CASE(256, 8, 4) SVM_DSMO_CASE(512, 4, 4)
  SVM_DSMO_CASE(512, 8, 4)
#undef SVM_DSMO_CASE
  set_error("dsmo: no kernel for NT=%d E=%d RPL=%d", sh.NT, sh.E, sh.RPL);
  return SVM_ERR_INTERNAL;
}

double ms_between(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

void hipck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw CascadeError(std::string(what) + ": " + hipGetErrorString(e));
}
void svck(int rc, const char* what) {
  if (rc != SVM_OK) throw CascadeError(std::string(what) + ": " + svm_last_error());
}

// Grow-only device allocation on one GPU (contents not preserved when it grows).
struct DBuf {
  void* p = nullptr;
  size_t bytes = 0;
  template <class T = void>
  T* ensure(size_t b) {
    if (b > bytes) {
      if (p) (void)hipFree(p);
      p = nullptr;
      bytes = 0;
      hipck(hipMalloc(&p, std::max<size_t>(b, 256)), "hipMalloc");
      bytes = std::max<size_t>(b, 256);
    }
    return static_cast<T*>(p);
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

struct Dev {
  int device = 0;
  void* ctx = nullptr;  // svmd context: the stream and its ordering helpers
  hipStream_t s = nullptr;
  DBuf X, y, alpha, f, st, err, trace, mm, mmscratch, Q, N0, WN, stw, aux;
  std::vector<int> teams;  // teams this GPU runs
  std::vector<void*> extra;
};

struct Team {
  int dev = 0;
  DBuf slab;
  int64_t ldw = 0, col0 = 0, ncols = 0;
  unsigned long long* uc = nullptr;  // receive array (uncached fine-grained HBM of its GPU)
};

// Host barrier of the device threads of one fit (generation counted, honours the abort token).
class HostBarrier {
 public:
  explicit HostBarrier(int n) : n_(n) {}
  void wait(const AbortToken& tok, double timeout_s) {
    std::unique_lock<std::mutex> lk(mu_);
    const uint64_t g = gen_;
    if (++waiting_ == n_) {
      waiting_ = 0;
      ++gen_;
      cv_.notify_all();
      return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    while (gen_ == g) {
      cv_.wait_for(lk, std::chrono::milliseconds(10));
      if (gen_ != g) break;
      if (tok.raised()) throw CascadeAborted("dsmo: another device failed");
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
        throw TransportError("dsmo: device threads did not meet at the launch barrier");
    }
  }

 private:
  int n_, waiting_ = 0;
  uint64_t gen_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
};

struct Group {
  int P = 0;
  bool rehearsal = false;
  int rank = -1;  // >= 0: one team of a per-process solve (its peers' arrays opened over IPC)
  double timeout_s = 60.0;
  std::vector<std::unique_ptr<Dev>> dev;
  std::vector<Team> team;
  std::unique_ptr<RankPool> pool;
  std::vector<unsigned long long*> uc_all;  // per team
  std::vector<void*> ipc_opened;            // peers' arrays mapped into this process
  bool connected = false;
  uint32_t epoch = 1;
  std::mutex mu;
  ~Group() {
    pool.reset();
    if (!dev.empty()) (void)hipSetDevice(dev[0]->device);
    for (void* q : ipc_opened) (void)hipIpcCloseMemHandle(q);
    for (auto& t : team) {
      if (t.dev < 0) continue;
      (void)hipSetDevice(dev[size_t(t.dev)]->device);
      t.slab.release();
      if (t.uc) (void)hipFree(t.uc);
    }
    for (auto& d : dev) {
      (void)hipSetDevice(d->device);
      for (DBuf* b : {&d->X, &d->y, &d->alpha, &d->f, &d->st, &d->err, &d->trace, &d->mm, &d->mmscratch, &d->Q,
                      &d->N0, &d->WN, &d->stw, &d->aux})
        b->release();
      if (d->ctx) svmd_destroy(d->ctx);
    }
  }
};

struct FitIn {
  const void* X;
  bool u8;
  const int32_t* y;
  int64_t n, d;
  svm_params p;
  int64_t* trace;
  int64_t tcap;
};

struct DevOut {
  std::vector<SmoState> st;  // per team of this GPU
  unsigned err = 0;
  double upload_ms = 0, gram_ms = 0, smo_ms = 0, total_ms = 0;
  Shape shape;
  std::vector<double> mnmx;  // column min then max (2d)
};

// Per-GPU state of one fit between prepare() and solve().
struct Prepared {
  Shape sh;
  QRows q{};
  DsmoArgs a{};
  int64_t* trd = nullptr;
  std::chrono::steady_clock::time_point t0, t_up, t_gram;
};

// Rows, labels, column statistics, exact-integer quantisation, this GPU's slabs and the cold start,
// synchronised (every GPU then launches at once).
void prepare(Group& g, int di, const FitIn& in, DevOut& out, Prepared& pr) {
  Dev& D = *g.dev[size_t(di)];
  hipck(hipSetDevice(D.device), "hipSetDevice");
  hipStream_t s = D.s;
  const int64_t n = in.n, d = in.d;
  pr.t0 = std::chrono::steady_clock::now();
  if (!in.u8) throw CascadeError("dsmo: needs uint8 pixel rows (the exact-integer Gram); use the cascade otherwise");
  // ---- rows and labels (every GPU holds all rows: slabs need them, K12 reads any pair)
  auto* Xd = D.X.ensure<uint8_t>(size_t(n) * size_t(d));
  auto* yd = D.y.ensure<int32_t>(size_t(n) * 4);
  auto* ad = D.alpha.ensure<double>(size_t(n) * 8);
  auto* fd = D.f.ensure<double>(size_t(n) * 8);
  auto* std_ = D.st.ensure<SmoState>(sizeof(SmoState) * kMaxPeers);
  auto* errd = D.err.ensure<unsigned>(256);
  hipck(hipMemcpyAsync(Xd, in.X, size_t(n) * size_t(d), hipMemcpyHostToDevice, s), "H2D rows");
  hipck(hipMemcpyAsync(yd, in.y, size_t(n) * 4, hipMemcpyHostToDevice, s), "H2D labels");
  // ---- column min / max (identical on every GPU: same bytes, deterministic kernel)
  auto* mm = D.mm.ensure<double>(size_t(2) * size_t(d) * 8);
  const size_t scratch = size_t(2) * size_t(d) * 2048;
  svck(launch_minmax_u8(s, Xd, n, d, mm, mm + d, D.mmscratch.ensure<double>(scratch * 8), scratch), "minmax");
  std::vector<double> mmh(size_t(2 * d));
  hipck(hipMemcpyAsync(mmh.data(), mm, size_t(2 * d) * 8, hipMemcpyDeviceToHost, s), "D2H min/max");
  hipck(hipStreamSynchronize(s), "sync");
  out.mnmx = mmh;
  pr.t_up = std::chrono::steady_clock::now();
  // ---- exact-integer quantisation from the bytes, then this GPU's slabs
  QuantPlan P;
  if (!plan_quant(mmh.data(), mmh.data() + d, d, &P) || P.kq > 32 * 128)
    throw CascadeError("dsmo: the rows are not integer pixels (no exact-integer plan)");
  auto* Q = D.Q.ensure<int8_t>(size_t(n) * size_t(P.kq));
  auto* N0 = D.N0.ensure<int32_t>(size_t(n) * 4);
  auto* WN = D.WN.ensure<double>(size_t(n) * 8);
  auto* stw = D.stw.ensure<double>(P.step_w.size() * 8);
  bool ok = false;
  svck(quantize_u8_rows(s, Xd, n, d, mmh.data(), mmh.data() + d, P, D.aux.ensure(quantize_u8_aux_bytes(P)), Q, N0, WN,
                        &ok),
       "quantise");
  if (!ok) throw CascadeError("dsmo: a row failed the exact-integer quantisation check");
  hipck(hipMemcpyAsync(stw, P.step_w.data(), P.step_w.size() * 8, hipMemcpyHostToDevice, s), "H2D step weights");
  int ncu = 0;
  hipck(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, D.device), "attribute");
  if (!dsmo_shape(n, g.P, ncu, g.rehearsal, &pr.sh)) throw CascadeError("dsmo: no team shape for this n and P");
  out.shape = pr.sh;
  for (int t = 0; t < g.P; ++t) {  // every team's column range (slabs only for this GPU's teams)
    Team& T = g.team[size_t(t)];
    T.col0 = std::min<int64_t>(n, int64_t(t) * pr.sh.W);
    T.ncols = std::min<int64_t>(n, T.col0 + pr.sh.W) - T.col0;
    T.ldw = pr.sh.W;
  }
  check_plan(n, g.P, ncu, g.rehearsal, pr.sh);
  for (int t : D.teams) {
    Team& T = g.team[size_t(t)];
    // the slab is read as slab[i * ldw + (j - col0)], i < n: it spans n full rows of ldw >= ncols
    const size_t slab_bytes = size_t(n) * size_t(T.ldw) * 8;
    double* slab = T.slab.ensure<double>(slab_bytes);
    if (T.slab.bytes < slab_bytes || T.ldw < T.ncols) throw CascadeError("dsmo: slab smaller than its index space");
    if (T.ncols > 0) svck(launch_igram_slab(s, Q, N0, WN, stw, n, T.col0, T.ncols, P, in.p.gamma, slab, T.ldw), "slab");
  }
  hipLaunchKernelGGL(dsmo_init_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, yd, ad, fd, n, std_, kMaxPeers);
  hipck(hipGetLastError(), "init kernel");
  hipck(hipMemsetAsync(errd, 0, 256, s), "memset");
  const bool has0 = std::find(D.teams.begin(), D.teams.end(), 0) != D.teams.end();
  pr.trd = (in.tcap > 0 && has0) ? D.trace.ensure<int64_t>(size_t(in.tcap) * 16) : nullptr;
  hipck(hipStreamSynchronize(s), "sync");
  pr.t_gram = std::chrono::steady_clock::now();
  for (int t = 0; t < g.P; ++t) {  // a peer's slab pointer is never dereferenced here (own team only)
    const Team& T = g.team[size_t(t)];
    pr.a.team[t] = DsmoTeam{T.slab.as<double>(), T.ldw, T.col0};
    pr.a.px.arr[t] = g.uc_all[size_t(t)];
  }
  pr.a.px.n = g.P;
  pr.a.teams = g.P;
  pr.a.Gt = pr.sh.Gt;
  pr.a.team_base = D.teams.front();
  pr.a.epoch0 = g.epoch;
  pr.q.Q = Q;
  pr.q.N0 = N0;
  pr.q.WN = WN;
  pr.q.step_w = stw;
  pr.q.kq = P.kq;
  pr.q.main_step0 = P.main0 / 32;
  pr.q.w0 = P.w0;
}

// Launch this GPU's team(s), wait, and copy the state, the error word and its alpha slice back.
void solve(Group& g, int di, const FitIn& in, double* alpha_out, DevOut& out, Prepared& pr) {
  Dev& D = *g.dev[size_t(di)];
  hipck(hipSetDevice(D.device), "hipSetDevice");
  hipStream_t s = D.s;
  {
    TraceRange tr("svm355:dsmo");
    svck(launch_dsmo(s, pr.sh, int(D.teams.size()) * pr.sh.Gt, pr.a, pr.q, -in.p.gamma, D.y.as<int32_t>(),
                     D.alpha.as<double>(), D.f.as<double>(), in.n, D.st.as<SmoState>(), in.p, pr.trd,
                     pr.trd ? in.tcap : 0, D.err.as<unsigned>()),
         "dsmo launch");
    out.st.resize(D.teams.size());
    std::vector<SmoState> sth(static_cast<size_t>(kMaxPeers));
    hipck(hipMemcpyAsync(sth.data(), D.st.as<SmoState>(), sizeof(SmoState) * kMaxPeers, hipMemcpyDeviceToHost, s),
          "D2H state");
    hipck(hipMemcpyAsync(&out.err, D.err.as<unsigned>(), 4, hipMemcpyDeviceToHost, s), "D2H err");
    for (size_t k = 0; k < D.teams.size(); ++k) {
      const Team& T = g.team[size_t(D.teams[k])];
      if (T.ncols > 0)
        hipck(hipMemcpyAsync(alpha_out + T.col0, D.alpha.as<double>() + T.col0, size_t(T.ncols) * 8,
                             hipMemcpyDeviceToHost, s),
              "D2H alpha");
    }
    if (pr.trd) hipck(hipMemcpyAsync(in.trace, pr.trd, size_t(in.tcap) * 16, hipMemcpyDeviceToHost, s), "D2H trace");
    hipck(hipStreamSynchronize(s), "sync");
    for (size_t k = 0; k < D.teams.size(); ++k) out.st[k] = sth[size_t(D.teams[k])];
  }
  const auto t_end = std::chrono::steady_clock::now();
  out.upload_ms = ms_between(pr.t0, pr.t_up);
  out.gram_ms = ms_between(pr.t_up, pr.t_gram);
  out.smo_ms = ms_between(pr.t_gram, t_end);
  out.total_ms = ms_between(pr.t0, t_end);
}

void dev_fit(Group& g, int di, const FitIn& in, double* alpha_out, DevOut& out, HostBarrier& bar,
             const AbortToken& tok) {
  Prepared pr;
  prepare(g, di, in, out, pr);
  bar.wait(tok, g.timeout_s);  // every GPU launches once all are ready (the spins absorb the rest)
  solve(g, di, in, alpha_out, out, pr);
}

// Result of the teams this call drove: they ran the identical update sequence, so their states must
// agree bit for bit.
int finish(Group& g, const std::vector<DevOut>& outs, const svm_params& p, const double* alpha_out, int64_t n,
           int64_t d, std::chrono::steady_clock::time_point t0, svm_result* r, double* timing_out, int32_t* shape_out,
           double* mn_out, double* mx_out) {
  const SmoState& s0 = outs[0].st[0];
  for (size_t di = 0; di < outs.size(); ++di) {
    if (outs[di].err) {
      set_error("dsmo: GPU %d: a workgroup timed out waiting for a peer record (exchange failed)",
                g.dev[di]->device);
      return SVM_ERR_DEVICE;
    }
    for (const SmoState& s : outs[di].st)
      if (s.num_iter != s0.num_iter || s.b_high != s0.b_high || s.b_low != s0.b_low || s.stop != s0.stop) {
        set_error("dsmo: teams disagree (iterations %lld vs %lld)", (long long)s.num_iter, (long long)s0.num_iter);
        return SVM_ERR_INTERNAL;
      }
  }
  if (!s0.stop) {
    set_error("dsmo: solver did not stop");
    return SVM_ERR_INTERNAL;
  }
  if (r) {
    r->iterations = s0.num_iter;
    r->b_high = s0.b_high;
    r->b_low = s0.b_low;
    r->b = (s0.b_high + s0.b_low) / 2;
    r->stop_reason = s0.stop;
    r->reserved = 0;
    int64_t c = 0;  // this call's slices only (a per-process rank counts its own)
    for (const auto& D : g.dev)
      for (int t : D->teams) {
        const Team& T = g.team[size_t(t)];
        for (int64_t i = T.col0; i < T.col0 + T.ncols; ++i) c += alpha_out[i] > p.sv_tol;
      }
    r->n_sv = c;
    r->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  if (timing_out) {  // slowest GPU per phase: upload+minmax, quantise+slabs, solve, total
    double mx[4] = {0, 0, 0, 0};
    for (const DevOut& o : outs) {
      mx[0] = std::max(mx[0], o.upload_ms);
      mx[1] = std::max(mx[1], o.gram_ms);
      mx[2] = std::max(mx[2], o.smo_ms);
      mx[3] = std::max(mx[3], o.total_ms);
    }
    std::copy(mx, mx + 4, timing_out);
  }
  if (mn_out) std::copy(outs[0].mnmx.begin(), outs[0].mnmx.begin() + d, mn_out);
  if (mx_out) std::copy(outs[0].mnmx.begin() + d, outs[0].mnmx.end(), mx_out);
  if (shape_out) {
    const Shape& sh = outs[0].shape;
    shape_out[0] = sh.NT;
    shape_out[1] = sh.E;
    shape_out[2] = sh.Gt;
    shape_out[3] = sh.RPL;
  }
  return SVM_OK;
}

// Advances the group's epoch past everything a solve may have used (max_iter + 2 epochs), whatever
// happened: a record left by an aborted solve can never match a later epoch.
struct EpochAdvance {
  Group* g;
  int64_t span;
  ~EpochAdvance() { g->epoch += uint32_t(std::min<int64_t>(span, int64_t(1) << 30)); }
};

int maybe_reset_epochs(Group& g) {
  if (g.epoch <= (1u << 31)) return SVM_OK;
  for (const Team& T : g.team) {  // far from wrapping: restart the tags on zeroed arrays
    if (T.dev < 0) continue;
    (void)hipSetDevice(g.dev[size_t(T.dev)]->device);
    if (hipMemset(T.uc, 0, kUcBytes) != hipSuccess) return SVM_ERR_DEVICE;
  }
  g.epoch = 1;
  return SVM_OK;
}

unsigned long long* alloc_uc(int device) {
  hipck(hipSetDevice(device), "hipSetDevice");
  void* p = nullptr;
  hipck(hipExtMallocWithFlags(&p, kUcBytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
  hipck(hipMemset(p, 0, kUcBytes), "hipMemset");  // tag 0 = no epoch
  hipck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return static_cast<unsigned long long*>(p);
}

Group* create_group(int P, bool rehearsal, double timeout_s) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  if (P < 1 || P > kMaxPeers) throw CascadeError("dsmo: 1 <= P <= " + std::to_string(kMaxPeers));
  if (ndev < 1) throw CascadeError("dsmo: no HIP device visible");
  if (!rehearsal && P > ndev)
    throw CascadeError("dsmo: " + std::to_string(P) + " GPUs requested, " + std::to_string(ndev) + " visible");
  auto g = std::make_unique<Group>();
  g->P = P;
  g->rehearsal = rehearsal;
  g->timeout_s = timeout_s > 0 ? timeout_s : 60.0;
  const int nd = rehearsal ? 1 : P;
  for (int i = 0; i < nd; ++i) {
    auto D = std::make_unique<Dev>();
    D->device = i;
    D->ctx = svmd_create(i);
    if (!D->ctx) throw CascadeError(std::string("svmd_create: ") + svm_last_error());
    D->s = static_cast<DeviceCtx*>(D->ctx)->stream;
    g->dev.push_back(std::move(D));
  }
  // Peer access between every pair of GPUs (remote stores into the peers' receive arrays).
  for (int i = 0; i < nd && nd > 1; ++i) {
    hipck(hipSetDevice(i), "hipSetDevice");
    for (int j = 0; j < nd; ++j) {
      if (i == j) continue;
      int can = 0;
      hipck(hipDeviceCanAccessPeer(&can, i, j), "hipDeviceCanAccessPeer");
      if (!can) throw CascadeError("dsmo: GPU " + std::to_string(i) + " cannot access GPU " + std::to_string(j));
      const hipError_t e = hipDeviceEnablePeerAccess(j, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) hipck(e, "hipDeviceEnablePeerAccess");
      (void)hipGetLastError();
    }
  }
  g->team.resize(size_t(P));
  for (int t = 0; t < P; ++t) {
    Team& T = g->team[size_t(t)];
    T.dev = rehearsal ? 0 : t;
    g->dev[size_t(T.dev)]->teams.push_back(t);
    T.uc = alloc_uc(g->dev[size_t(T.dev)]->device);
    g->uc_all.push_back(T.uc);
  }
  g->pool = std::make_unique<RankPool>(nd);
  g->connected = true;
  return g.release();
}

}  // namespace
}  // namespace svm355

using namespace svm355;

extern "C" {

SVM_API void* svmd_dsmo_create(int32_t world, int32_t rehearsal, double timeout_s) {
  try {
    return create_group(world, rehearsal != 0, timeout_s);
  } catch (const std::exception& e) {
    set_error("svmd_dsmo_create: %s", e.what());
    return nullptr;
  }
}

SVM_API void svmd_dsmo_destroy(void* h) { delete static_cast<Group*>(h); }

SVM_API int svmd_dsmo_fit(void* h, const void* X, int32_t u8, const int32_t* y, int64_t n, int64_t d,
                          const svm_params* pp, double* alpha_out, svm_result* r, double* timing_out,
                          int64_t* trace, int64_t trace_cap, int32_t* shape_out, double* mn_out, double* mx_out) {
  auto* g = static_cast<Group*>(h);
  if (!g || !X || !y || !alpha_out || n < 2 || d <= 0 || n >= int64_t(kSentinel)) {
    set_error("svmd_dsmo_fit: bad arguments");
    return SVM_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(g->mu);
  svm_params p;
  if (pp)
    p = *pp;
  else
    svm_default_params(&p);
  if (p.wss == 2) {
    set_error("svmd_dsmo_fit: the distributed solver is first-order (wss = 1)");
    return SVM_ERR_ARG;
  }
  const auto t0 = std::chrono::steady_clock::now();
  const int nd = int(g->dev.size());
  FitIn in{X, u8 != 0, y, n, d, p, trace, trace_cap};
  std::vector<DevOut> outs(static_cast<size_t>(nd));
  HostBarrier bar(nd);
  auto token = std::make_shared<AbortToken>();
  int rc = maybe_reset_epochs(*g);
  if (rc) return rc;
  EpochAdvance adv{g, p.max_iter + 4};
  try {
    g->pool->run(
        token, [&](int di) { dev_fit(*g, di, in, alpha_out, outs[size_t(di)], bar, *token); }, [](int) {});
  } catch (const std::exception& e) {
    set_error("svmd_dsmo_fit: %s", e.what());
    return SVM_ERR_DEVICE;
  }
  return finish(*g, outs, p, alpha_out, n, d, t0, r, timing_out, shape_out, mn_out, mx_out);
}

SVM_API int svmd_dsmo_world(void* h) { return h ? static_cast<Group*>(h)->P : 0; }

// The team plan for n points over P teams (ncu CUs per GPU; one_launch: all teams co-resident on one
// GPU): out = {NT, E, Gt, RPL, slice, W}.  No device needed (host checks / tests).
SVM_API int svmd_dsmo_plan(int64_t n, int32_t P, int32_t ncu, int32_t one_launch, int64_t* out) {
  try {
    Shape sh;
    if (!dsmo_shape(n, P, ncu, one_launch != 0, &sh)) {
      set_error("dsmo plan: no shape for n=%lld P=%d", (long long)n, P);
      return SVM_ERR_ARG;
    }
    check_plan(n, P, ncu, one_launch != 0, sh);
    const int64_t v[6] = {sh.NT, sh.E, sh.Gt, sh.RPL, sh.slice, sh.W};
    if (out) std::copy(v, v + 6, out);
    return SVM_OK;
  } catch (const std::exception& e) {
    set_error("%s", e.what());
    return SVM_ERR_ARG;
  }
}

// ---- one team per PROCESS (torchrun): the receive arrays are exchanged as IPC handles through the
// launcher (svmd_dsmo_rank_handle -> all-gather -> svmd_dsmo_rank_connect); a fit is prepare (rows,
// slabs), a barrier of the launcher, then solve (the launch), so every GPU starts together.
SVM_API void* svmd_dsmo_rank_create(int32_t device, int32_t world, int32_t rank, double timeout_s) {
  try {
    if (world < 1 || world > kMaxPeers || rank < 0 || rank >= world) throw CascadeError("bad world / rank");
    auto g = std::make_unique<Group>();
    g->P = world;
    g->rank = rank;
    g->timeout_s = timeout_s > 0 ? timeout_s : 60.0;
    auto D = std::make_unique<Dev>();
    D->device = device;
    hipck(hipSetDevice(device), "hipSetDevice");
    D->ctx = svmd_create(device);
    if (!D->ctx) throw CascadeError(std::string("svmd_create: ") + svm_last_error());
    D->s = static_cast<DeviceCtx*>(D->ctx)->stream;
    D->teams.push_back(rank);
    g->dev.push_back(std::move(D));
    g->team.resize(size_t(world));
    for (int t = 0; t < world; ++t) g->team[size_t(t)].dev = t == rank ? 0 : -1;
    g->team[size_t(rank)].uc = alloc_uc(device);
    g->uc_all.assign(size_t(world), nullptr);
    g->uc_all[size_t(rank)] = g->team[size_t(rank)].uc;
    return g.release();
  } catch (const std::exception& e) {
    set_error("svmd_dsmo_rank_create: %s", e.what());
    return nullptr;
  }
}

SVM_API int64_t svmd_dsmo_handle_bytes(void) { return int64_t(sizeof(hipIpcMemHandle_t)); }

SVM_API int svmd_dsmo_rank_handle(void* h, uint8_t* out, int64_t cap) {
  auto* g = static_cast<Group*>(h);
  if (!g || g->rank < 0 || !out || cap < int64_t(sizeof(hipIpcMemHandle_t))) {
    set_error("svmd_dsmo_rank_handle: bad arguments");
    return SVM_ERR_ARG;
  }
  hipIpcMemHandle_t hd;
  (void)hipSetDevice(g->dev[0]->device);
  const hipError_t e = hipIpcGetMemHandle(&hd, g->team[size_t(g->rank)].uc);
  if (e != hipSuccess) {
    set_error("hipIpcGetMemHandle: %s", hipGetErrorString(e));
    return SVM_ERR_DEVICE;
  }
  std::memcpy(out, &hd, sizeof(hd));
  return SVM_OK;
}

// handles: world entries of svmd_dsmo_handle_bytes() each, in rank order (this rank's is ignored).
SVM_API int svmd_dsmo_rank_connect(void* h, const uint8_t* handles) {
  auto* g = static_cast<Group*>(h);
  if (!g || g->rank < 0 || !handles) {
    set_error("svmd_dsmo_rank_connect: bad arguments");
    return SVM_ERR_ARG;
  }
  (void)hipSetDevice(g->dev[0]->device);
  for (int t = 0; t < g->P; ++t) {
    if (t == g->rank) continue;
    hipIpcMemHandle_t hd;
    std::memcpy(&hd, handles + size_t(t) * sizeof(hd), sizeof(hd));
    void* q = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&q, hd, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      set_error("hipIpcOpenMemHandle (rank %d's receive array): %s", t, hipGetErrorString(e));
      return SVM_ERR_DEVICE;
    }
    g->ipc_opened.push_back(q);
    g->uc_all[size_t(t)] = static_cast<unsigned long long*>(q);
  }
  g->connected = true;
  return SVM_OK;
}

namespace {
struct RankFit {
  FitIn in;
  std::vector<DevOut> outs;
  Prepared pr;
  std::chrono::steady_clock::time_point t0;
  bool ready = false;
};
std::mutex g_rank_mu;
std::map<void*, std::unique_ptr<RankFit>> g_rank_fits;  // pending fit per rank handle
}  // namespace

SVM_API int svmd_dsmo_rank_prepare(void* h, const void* X, int32_t u8, const int32_t* y, int64_t n, int64_t d,
                                   const svm_params* pp) {
  auto* g = static_cast<Group*>(h);
  if (!g || g->rank < 0 || !g->connected || !X || !y || n < 2 || d <= 0 || n >= int64_t(kSentinel)) {
    set_error("svmd_dsmo_rank_prepare: bad arguments (or not connected)");
    return SVM_ERR_ARG;
  }
  svm_params p;
  if (pp)
    p = *pp;
  else
    svm_default_params(&p);
  if (p.wss == 2) {
    set_error("svmd_dsmo_rank_prepare: the distributed solver is first-order (wss = 1)");
    return SVM_ERR_ARG;
  }
  auto f = std::make_unique<RankFit>();
  f->t0 = std::chrono::steady_clock::now();
  f->in = FitIn{X, u8 != 0, y, n, d, p, nullptr, 0};
  f->outs.resize(1);
  try {
    int rc = maybe_reset_epochs(*g);
    if (rc) return rc;
    prepare(*g, 0, f->in, f->outs[0], f->pr);
  } catch (const std::exception& e) {
    set_error("svmd_dsmo_rank_prepare: %s", e.what());
    return SVM_ERR_DEVICE;
  }
  f->ready = true;
  std::lock_guard<std::mutex> lk(g_rank_mu);
  g_rank_fits[h] = std::move(f);
  return SVM_OK;
}

// Collective after a barrier of every rank's prepare: this rank's alpha slice into alpha_out (n
// doubles; other entries untouched); range_out (optional, 2 int64): the slice [col0, col0 + ncols).
SVM_API int svmd_dsmo_rank_solve(void* h, double* alpha_out, svm_result* r, double* timing_out, int32_t* shape_out,
                                 double* mn_out, double* mx_out, int64_t* range_out) {
  auto* g = static_cast<Group*>(h);
  std::unique_ptr<RankFit> f;
  {
    std::lock_guard<std::mutex> lk(g_rank_mu);
    auto it = g_rank_fits.find(h);
    if (it != g_rank_fits.end()) {
      f = std::move(it->second);
      g_rank_fits.erase(it);
    }
  }
  if (!g || !f || !f->ready || !alpha_out) {
    set_error("svmd_dsmo_rank_solve: no prepared fit");
    return SVM_ERR_ARG;
  }
  EpochAdvance adv{g, f->in.p.max_iter + 4};
  try {
    solve(*g, 0, f->in, alpha_out, f->outs[0], f->pr);
  } catch (const std::exception& e) {
    set_error("svmd_dsmo_rank_solve: %s", e.what());
    return SVM_ERR_DEVICE;
  }
  if (range_out) {
    const Team& T = g->team[size_t(g->rank)];
    range_out[0] = T.col0;
    range_out[1] = T.ncols;
  }
  return finish(*g, f->outs, f->in.p, alpha_out, f->in.n, f->in.d, f->t0, r, timing_out, shape_out, mn_out, mx_out);
}

}  // extern "C"

SVMD_TU_WARM(dsmo)
