// CpuBackend: the cascade's rows in host memory and every solve on the C++ oracle SMO
// (smo_cpu.cpp, the reference arithmetic of mpi_svm_main3.cpp:155-290 with init = false).  Rows
// are stored unpadded (ld = d), which is exactly the oracle's input layout, so a solve reads the
// assembled set in place.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cascade.h"

namespace svm355 {
namespace {

class CpuBackend final : public Backend {
 public:
  const char* name() const override { return "cpu"; }
  int64_t ld(int64_t d) const override { return d; }
  void* alloc(int64_t bytes) override {
    const size_t sz = (size_t(std::max<int64_t>(bytes, 1)) + 63) & ~size_t(63);
    void* p = std::aligned_alloc(64, sz);
    if (!p) throw CascadeError("host allocation of " + std::to_string(bytes) + " bytes failed");
    return p;
  }
  void free(void* p) override { std::free(p); }
  void h2d(void* dst, const void* src, int64_t bytes) override {
    if (bytes > 0) std::memcpy(dst, src, size_t(bytes));
  }
  void d2h(void* dst, const void* src, int64_t bytes) override {
    if (bytes > 0) std::memcpy(dst, src, size_t(bytes));
  }
  void sync() override {}
  void upload_rows(const void* X, bool u8, int64_t n, int64_t d, double* dst) override {
    if (!u8) {
      std::memcpy(dst, X, size_t(n * d) * 8);
      return;
    }
    const auto* p = static_cast<const uint8_t*>(X);
    for (int64_t i = 0; i < n * d; ++i) dst[i] = double(p[i]);
  }
  void minmax(const double* X, int64_t n, int64_t d, double* mn, double* mx) override {
    if (n == 0) {
      for (int64_t j = 0; j < d; ++j) {
        mn[j] = __builtin_inf();
        mx[j] = -__builtin_inf();
      }
      return;
    }
    check(svm_minmax(X, n, d, mn, mx), "svm_minmax");
  }
  void scale(double* X, int64_t n, int64_t d, const double* mn, const double* mx) override {
    check(svm_scale(X, n, d, mn, mx), "svm_scale");
  }
  void assemble(const Segment& s, int64_t ld, DSet& o, int64_t off) override {
    const int64_t m = s.rows();
    auto* X = o.X.as<double>();
    auto* y = o.y.as<int32_t>();
    auto* a = o.a.as<double>();
    auto* id = o.id.as<int64_t>();
    for (int64_t i = 0; i < m; ++i) {
      const int64_t src = s.idx ? (*s.idx)[size_t(i)] : i, dst = off + i;
      if (s.set) {
        std::memcpy(X + dst * ld, s.set->X.as<double>() + src * ld, size_t(ld) * 8);
        y[dst] = s.set->y.as<int32_t>()[src];
        a[dst] = s.zero_alpha ? 0.0 : s.set->a.as<double>()[src];
        id[dst] = s.set->id.as<int64_t>()[src];
      } else {
        const double* r = s.rec + src * (ld + 3);
        std::memcpy(X + dst * ld, r, size_t(ld) * 8);
        y[dst] = int32_t(r[ld]);
        a[dst] = s.zero_alpha ? 0.0 : r[ld + 1];
        id[dst] = int64_t(r[ld + 2]);
      }
    }
  }
  void pack(const DSet& S, int64_t ld, double* rec) override {
    for (int64_t i = 0; i < S.k; ++i) {
      double* r = rec + i * (ld + 3);
      std::memcpy(r, S.X.as<double>() + i * ld, size_t(ld) * 8);
      r[ld] = double(S.y.as<int32_t>()[i]);
      r[ld + 1] = S.a.as<double>()[i];
      r[ld + 2] = double(S.id.as<int64_t>()[i]);
    }
  }
  void record_ids(const double* rec, int64_t k, int64_t ld, int64_t* ids) override {
    for (int64_t i = 0; i < k; ++i) ids[i] = int64_t(rec[i * (ld + 3) + ld + 2]);
  }
  static constexpr double kDenseKBudget = 4.0 * (1ull << 30);  // bytes of one solve's dense kernel matrix
  SolveStats solve(DSet& S, int64_t d, const svm_params& p, const double*, const double*, int solver,
                   int64_t) override {
    svm_result r{};
    // the decomposition oracle holds the set's dense k x k kernel matrix: above the budget (a 60k
    // single-rank set would need 28.8 GB) the solve streams rows with the pairwise oracle instead, and
    // the log says so (solver 0)
    if (solver == 1 && S.k >= 2 && double(S.k) * double(S.k) * 8.0 > kDenseKBudget) solver = 0;
    if (solver == 1 && S.k >= 2) {
      // the decomposition oracle (decomp_cpu.cpp) on the set's kernel matrix (the reference's direct
      // RBF, svm_rbf_matrix), warm started from S.a
      std::vector<double> K;
      try {
        K.resize(size_t(S.k) * size_t(S.k));
      } catch (const std::bad_alloc&) {
        throw CascadeError("CPU backend: no memory for the " + std::to_string(S.k) + " x " + std::to_string(S.k) +
                           " kernel matrix of a decomposition solve");
      }
      check(svm_rbf_matrix(S.X.as<double>(), S.k, S.X.as<double>(), S.k, d, p.gamma, K.data(), p.n_threads),
            "svm_rbf_matrix");
      int64_t ds[SVM_DECOMP_STATS] = {};
      check(svm_decomp_train_gram(K.data(), S.k, S.y.as<int32_t>(), S.k, S.a.as<double>(), 1, &p, 1024, 0.1, 3, &r, ds,
                                  nullptr),
            "svm_decomp_train_gram");
      SolveStats st{r.iterations, r.b, r.stop_reason, 0.0};
      st.solver = 1;
      st.outer = ds[0];
      return st;
    }
    check(svm_smo_train(S.X.as<double>(), S.y.as<int32_t>(), S.k, d, S.a.as<double>(), 1, &p, &r, nullptr, 0),
          "svm_smo_train");
    return SolveStats{r.iterations, r.b, r.stop_reason, 0.0};
  }

 private:
  static void check(int rc, const char* what) {
    if (rc != SVM_OK) throw CascadeError(std::string(what) + ": " + svm_last_error());
  }
};

}  // namespace

std::unique_ptr<Backend> make_cpu_backend() { return std::make_unique<CpuBackend>(); }

}  // namespace svm355
