// svm_serial — serial CPU SMO trainer/evaluator (the reference's code/main3.cpp program).
//
// Same pipeline, timing scopes and stdout lines as main3.cpp:306-417:
//   read train CSV (untimed) -> [timer] min/max + scale -> SMO -> read + scale test -> SV count
//   [end "training"] -> predict over SVs -> [end "prediction"].
// Every compile-time constant of the reference is a flag (cli_common.h).  --threads > 1 parallelises
// the O(n) loops without changing any result (the serial baseline is --threads 1, the default).
#include <cstdio>

#include "cli_common.h"

int main(int argc, char** argv) {
  cli::Options o;
  if (!cli::parse(argc, argv, o, 1)) return 2;

  cli::Data tr;
  if (!cli::load_split(o, true, tr)) return 1;
  printf("n = %lld\n", tr.n);
  printf("n_features = %lld\n", tr.d);
  if (tr.n == 0) {
    fprintf(stderr, "Error: No data read from file.\n");
    return 1;
  }
  const long long n = tr.n, d = tr.d;
  std::vector<double> mn(static_cast<size_t>(d)), mx(static_cast<size_t>(d));

  const auto t_start = std::chrono::steady_clock::now();
  svm_minmax(tr.X.data(), n, d, mn.data(), mx.data());
  svm_scale(tr.X.data(), n, d, mn.data(), mx.data());

  std::vector<double> alpha(size_t(n), 0.0);
  svm_result r{};
  o.p.verbose = 1;  // stderr stop messages as in the reference
  if (svm_smo_train(tr.X.data(), tr.y.data(), n, d, alpha.data(), 0, &o.p, &r, nullptr, 0) != SVM_OK) {
    fprintf(stderr, "%s\n", svm_last_error());
    return 1;
  }
  printf("number of iterations: %lld\n", (long long)r.iterations);
  printf("b = %.15f\n", r.b);
  printf("(b_high - b_low)/2*1e10 = %.15f\n", (r.b_high - r.b_low) / 2 * 1e10);

  // Test read + scale sit inside the reference's "training" timer (main3.cpp:350-355).
  cli::Data te;
  if (!cli::load_split(o, false, te)) return 1;
  const long long m = te.n;
  if (m > 0) svm_scale(te.X.data(), m, d, mn.data(), mx.data());

  std::vector<int64_t> sv(static_cast<size_t>(n));
  const int64_t nsv = svm_sv_indices(alpha.data(), n, o.p.sv_tol, sv.data());
  sv.resize(size_t(nsv));
  printf("Final SV count = %lld\n", (long long)nsv);
  const auto t_end1 = std::chrono::steady_clock::now();

  // Predict over the SVs only (main3.cpp:391-402): curr = -b + sum alpha y K; y = curr > 0 ? 1 : -1.
  std::vector<double> Xs(static_cast<size_t>(nsv * d)), as(static_cast<size_t>(nsv));
  std::vector<int32_t> ys(static_cast<size_t>(nsv));
  for (int64_t k = 0; k < nsv; ++k) {
    const int64_t j = sv[size_t(k)];
    std::copy(tr.X.begin() + j * d, tr.X.begin() + (j + 1) * d, Xs.begin() + k * d);
    ys[size_t(k)] = tr.y[size_t(j)];
    as[size_t(k)] = alpha[size_t(j)];
  }
  std::vector<double> dec(static_cast<size_t>(m));
  svm_decision(Xs.data(), ys.data(), as.data(), nsv, te.X.data(), m, d, o.p.gamma, r.b, dec.data(), o.p.n_threads);
  long long correct = 0;
  for (long long i = 0; i < m; ++i) correct += ((dec[size_t(i)] > 0 ? 1 : -1) == te.y[size_t(i)]);
  printf("Test accuracy = %.15f (%lld/%lld)\n", m ? double(correct) / double(m) : 0.0, correct, m);
  const auto t_end2 = std::chrono::steady_clock::now();

  const double train_ms = cli::ms_between(t_start, t_end1), pred_ms = cli::ms_between(t_end1, t_end2);
  printf("Training time: %lld ms\n", (long long)train_ms);
  printf("Prediction time: %lld ms\n", (long long)pred_ms);
  printf("Total Runtime: %lld ms\n", (long long)(train_ms + pred_ms));

  if (!o.model_dir.empty()) {
    std::vector<int32_t> lab(ys);
    if (svm_model_save(o.model_dir.c_str(), sv.data(), lab.data(), as.data(), nsv, r.b) != SVM_OK)
      fprintf(stderr, "%s\n", svm_last_error());
  }
  cli::write_json(o.json, "svm_serial", o, n, d, r, correct, m, train_ms, pred_ms, train_ms + pred_ms, "");
  return 0;
}
