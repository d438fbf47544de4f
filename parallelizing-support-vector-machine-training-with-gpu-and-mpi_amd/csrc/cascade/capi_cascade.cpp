// C ABI of the cascade on the CPU oracle backend (thread ranks, loopback transport) and the result
// builder shared with the device library's entry points.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../core/internal.h"
#include "cascade_capi.h"

namespace svm355 {

CascadeConfig config_from(const svm_cascade_cfg* c) {
  svm_cascade_cfg d;
  svm_cascade_default_cfg(&d);
  if (!c) c = &d;
  CascadeConfig cfg;
  cfg.tree = c->tree != 0;
  cfg.max_rounds = c->max_rounds;
  cfg.params = c->params;
  cfg.log = c->log != 0;
  cfg.resume = c->resume != 0;
  cfg.checkpoint_dir = c->checkpoint_dir ? c->checkpoint_dir : "";
  cfg.fail_rank = c->fail_rank;
  cfg.fail_round = c->fail_round;
  cfg.fail_stall_s = c->fail_stall_s;
  cfg.solver = c->solver;
  return cfg;
}

std::vector<int64_t> partition_ids(int64_t n, int P, int r, int64_t* lo, int64_t* hi) {
  partition_bounds(n, P, r, lo, hi);
  std::vector<int64_t> ids(size_t(*hi - *lo));
  for (size_t i = 0; i < ids.size(); ++i) ids[i] = *lo + int64_t(i);
  return ids;
}

namespace {
template <class T>
T* dup(const std::vector<T>& v) {
  T* p = static_cast<T*>(std::malloc(std::max<size_t>(v.size(), 1) * sizeof(T)));
  if (!p) throw CascadeError("out of host memory");
  if (!v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
  return p;
}
}  // namespace

svm_cascade_out* build_cascade_out(const std::vector<const CascadeOutput*>& outs, Backend& B0, int world,
                                   int first_rank, const char* transport, const char* backend) {
  const CascadeOutput& R = *outs[0];
  auto* o = static_cast<svm_cascade_out*>(std::calloc(1, sizeof(svm_cascade_out)));
  if (!o) throw CascadeError("out of host memory");
  o->world = world;
  o->rank = first_rank;
  o->rounds = R.rounds;
  o->converged = R.converged ? 1 : 0;
  o->b = R.b;
  o->d = R.d;
  o->n_sv = int64_t(R.ids.size());
  o->ids = dup(R.ids);
  o->y = dup(R.y);
  o->alpha = dup(R.alpha);
  std::vector<double> rows(size_t(o->n_sv) * size_t(R.d));
  if (o->n_sv) {
    std::vector<double> wide(size_t(o->n_sv) * size_t(R.ld));
    B0.d2h(wide.data(), R.final_set.X.get(), o->n_sv * R.ld * 8);
    for (int64_t i = 0; i < o->n_sv; ++i)
      std::memcpy(&rows[size_t(i * R.d)], &wide[size_t(i * R.ld)], size_t(R.d) * 8);
  }
  o->sv_rows = dup(rows);
  o->mn = dup(R.mn);
  o->mx = dup(R.mx);
  o->n_hist = int64_t(R.sv_history.size());
  o->sv_history = dup(R.sv_history);
  o->round_ms = dup(R.round_ms);
  o->n_merged = int64_t(R.merged_history.size());
  o->merged_history = dup(R.merged_history);
  std::vector<double> solves, tms;
  for (const CascadeOutput* x : outs) {
    tms.push_back(x->train_ms);
    for (const SolveLog& s : x->solves)
      solves.insert(solves.end(), {double(s.rank), double(s.round), double(s.layer), double(s.rows),
                                   double(s.iterations), s.ms, s.b, double(s.stop), s.gram_ms,
                                   s.skipped ? 1.0 : 0.0, s.row_cache ? 1.0 : 0.0, s.solo_ms, double(s.solver),
                                   double(s.outer)});
  }
  static_assert(kNumPhases == sizeof(o->phase_ms) / sizeof(double), "svm_cascade_out.phase_ms size");
  std::copy(R.phase_ms, R.phase_ms + kNumPhases, o->phase_ms);
  o->n_solves = int64_t(solves.size() / SVM_CASCADE_SOLVE_COLS);
  o->solves = dup(solves);
  o->n_ranks = int64_t(tms.size());
  o->rank_train_ms = dup(tms);
  o->train_ms = tms.empty() ? 0.0 : *std::max_element(tms.begin(), tms.end());
  std::strncpy(o->transport, transport, sizeof(o->transport) - 1);
  std::strncpy(o->backend, backend, sizeof(o->backend) - 1);
  return o;
}

}  // namespace svm355

using namespace svm355;

extern "C" {

SVM_API void svm_cascade_default_cfg(svm_cascade_cfg* c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->tree = 0;
  c->max_rounds = 50;
  svm_default_params(&c->params);
  c->log = 0;
  c->resume = 0;
  c->checkpoint_dir = nullptr;
  c->comm_timeout_s = 600.0;
  c->fail_rank = -1;
  c->fail_round = -1;
  c->fail_stall_s = 0.0;
  c->solver = 0;
  c->reserved = 0;
}

SVM_API void svm_cascade_free(svm_cascade_out* o) {
  if (!o) return;
  for (void* p : {static_cast<void*>(o->ids), static_cast<void*>(o->y), static_cast<void*>(o->alpha),
                  static_cast<void*>(o->sv_rows), static_cast<void*>(o->mn), static_cast<void*>(o->mx),
                  static_cast<void*>(o->sv_history), static_cast<void*>(o->round_ms),
                  static_cast<void*>(o->merged_history), static_cast<void*>(o->solves),
                  static_cast<void*>(o->rank_train_ms)})
    std::free(p);
  std::free(o);
}

SVM_API svm_cascade_out* svm_cascade_fit_cpu(const double* X, const int32_t* y, int64_t n, int64_t d, int32_t world,
                                             const svm_cascade_cfg* c) {
  if (world < 1 || n < 0 || d <= 0 || (n && (!X || !y))) {
    set_error("svm_cascade_fit_cpu: bad arguments");
    return nullptr;
  }
  try {
    const CascadeConfig cfg = config_from(c);
    auto token = std::make_shared<AbortToken>();
    WaitPolicy wp{token, (c && c->comm_timeout_s > 0) ? c->comm_timeout_s : 600.0};
    auto group = std::make_shared<LoopbackGroup>(world, wp);
    std::vector<std::unique_ptr<Backend>> be(static_cast<size_t>(world));
    std::vector<std::unique_ptr<LoopbackTransport>> tr(static_cast<size_t>(world));
    for (int r = 0; r < world; ++r) {
      be[size_t(r)] = make_cpu_backend();
      tr[size_t(r)] = std::make_unique<LoopbackTransport>(group, r, be[size_t(r)].get());
    }
    std::vector<CascadeOutput> outs(static_cast<size_t>(world));
    run_rank_threads(
        world, token,
        [&](int r) {
          int64_t lo = 0, hi = 0;
          const std::vector<int64_t> ids = partition_ids(n, world, r, &lo, &hi);
          outs[size_t(r)] = run_cascade(*tr[size_t(r)], *be[size_t(r)], X + lo * d, false, y + lo, ids.data(), hi - lo,
                                        d, n, cfg);
        },
        [&](int r) { tr[size_t(r)]->abort(); });
    std::vector<const CascadeOutput*> ptrs;
    for (const auto& o : outs) ptrs.push_back(&o);
    return build_cascade_out(ptrs, *be[0], world, 0, "loopback", "cpu");
  } catch (const std::exception& e) {
    set_error("cascade: %s", e.what());
    return nullptr;
  }
}

}  // extern "C"
