// Shared command-line plumbing for the native CLIs (svm_serial, svm_gpu).
//
// The reference programs take no flags (every knob is a compile-time constant); these
// CLIs expose each knob with the reference default:
//   --dataset P      CSV prefix, reads P_train_data.csv / P_test_data.csv   (default mnist3)
//   --train F --test F   explicit CSV paths
//   --synthetic N[,M]    generate MNIST-shaped data instead (N train, M test rows; --seed S)
//   --n-limit N      train row limit (gpu_svm_main4.cu:489-490)
//   --C --gamma --tau --eps --sv-tol --max-iter --positive-label --threads
//   --model-dir D    write final_sv_{ids,labels,alphas}.txt and final_b.txt
//   --json F         machine-readable summary
//   --gram auto|fp64|int  (svm_gpu) RBF Gram path: exact-integer int8 MFMA for pixel data, or FP64 MFMA
//   --warmup W       (svm_gpu) untimed training runs first (steady-state timings)
//   --wss first|second  working-set selection: first order (the reference, default) or the opt-in
//                    second-order choice of the second index (Fan, Chen & Lin 2005)
#pragma once
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "svm355.h"

namespace cli {

struct Options {
  std::string dataset = "mnist3";
  std::string train, test, model_dir, json;
  long long synth_train = 0, synth_test = 0;
  unsigned long long seed = 2024;
  long long n_limit = -1;
  long long test_limit = -1;
  int positive_label = 1;
  svm_params p{};
  bool quiet = false;
  int gram_mode = 0;  // svm_gpu: 0 auto (exact-integer int8 MFMA Gram for pixel data), 1 fp64, 2 int
  int warmup = 0;     // svm_gpu: untimed training runs before the timed one
  int solver = 2;     // 1 working-set decomposition, 0 the pairwise SMO (the reference's trajectory, --solver
                      // smo), 2 auto (default): svm_gpu the decomposition, svm_cascade per solve (cascade.h)
};

inline void usage(const char* prog) {
  fprintf(stderr,
          "usage: %s [--dataset P | --train F --test F | --synthetic N[,M] [--seed S]] [--n-limit N]\n"
          "          [--C 10] [--gamma 0.00125] [--tau 1e-5] [--eps 1e-12] [--sv-tol 1e-8]\n"
          "          [--max-iter 100000] [--positive-label 1] [--threads T] [--model-dir D] [--json F]\n"
          "          [--gram auto|fp64|int] [--warmup W] [--wss first|second] [--solver auto|decomp|smo]\n",
          prog);
}

// Numeric option values parse whole or the run ends (exit 2), as argparse does: atof("1e-5x") would be
// 1e-5 and atoll("abc") a silent 0 (--synthetic abc read the default CSVs instead).
inline double parse_num(const char* what, const char* v) {
  char* end = nullptr;
  const double x = strtod(v, &end);
  if (end == v || *end != '\0') {
    fprintf(stderr, "invalid number for %s: '%s'\n", what, v);
    exit(2);
  }
  return x;
}

inline long long parse_int(const char* what, const char* v, bool until_comma = false) {
  char* end = nullptr;
  const long long x = strtoll(v, &end, 10);
  if (end == v || (*end != '\0' && !(until_comma && *end == ','))) {
    fprintf(stderr, "invalid integer for %s: '%s'\n", what, v);
    exit(2);
  }
  return x;
}

inline bool parse(int argc, char** argv, Options& o, int default_threads) {
  svm_default_params(&o.p);
  o.p.n_threads = default_threads;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&](const char* what) -> const char* {
      if (i + 1 >= argc) {
        fprintf(stderr, "missing value for %s\n", what);
        exit(2);
      }
      return argv[++i];
    };
    auto num = [&](const char* what) { return parse_num(what, next(what)); };
    auto count = [&](const char* what, const char* v, bool until_comma = false) {
      return parse_int(what, v, until_comma);
    };
    if (a == "--dataset") o.dataset = next("--dataset");
    else if (a == "--train") o.train = next("--train");
    else if (a == "--test") o.test = next("--test");
    else if (a == "--synthetic") {
      const char* v = next("--synthetic");
      o.synth_train = count("--synthetic", v, true);
      const char* c = strchr(v, ',');
      o.synth_test = c ? count("--synthetic", c + 1) : 10000;
      if (o.synth_train < 1 || o.synth_test < 0) {
        fprintf(stderr, "--synthetic N[,M] needs N >= 1, M >= 0\n");
        return false;
      }
    } else if (a == "--seed") o.seed = (unsigned long long)count("--seed", next("--seed"));
    else if (a == "--n-limit") o.n_limit = count("--n-limit", next("--n-limit"));
    else if (a == "--test-limit") o.test_limit = count("--test-limit", next("--test-limit"));
    else if (a == "--C") o.p.C = num("--C");
    else if (a == "--gamma") o.p.gamma = num("--gamma");
    else if (a == "--tau") o.p.tau = num("--tau");
    else if (a == "--eps") o.p.eps = num("--eps");
    else if (a == "--sv-tol") o.p.sv_tol = num("--sv-tol");
    else if (a == "--max-iter") o.p.max_iter = count("--max-iter", next("--max-iter"));
    else if (a == "--positive-label") o.positive_label = (int)count("--positive-label", next("--positive-label"));
    else if (a == "--threads") o.p.n_threads = (int)count("--threads", next("--threads"));
    else if (a == "--model-dir") o.model_dir = next("--model-dir");
    else if (a == "--json") o.json = next("--json");
    else if (a == "--quiet") o.quiet = true;
    else if (a == "--warmup") o.warmup = (int)count("--warmup", next("--warmup"));
    else if (a == "--gram") {
      const std::string g = next("--gram");
      if (g != "auto" && g != "fp64" && g != "int") {
        fprintf(stderr, "--gram must be auto, fp64 or int\n");
        return false;
      }
      o.gram_mode = g == "fp64" ? 1 : g == "int" ? 2 : 0;
    } else if (a == "--solver") {
      const std::string v = next("--solver");
      if (v != "smo" && v != "decomp" && v != "auto") {
        fprintf(stderr, "--solver must be smo, decomp or auto\n");
        return false;
      }
      o.solver = v == "decomp" ? 1 : v == "smo" ? 0 : 2;
    } else if (a == "--wss") {
      const std::string w = next("--wss");
      if (w != "first" && w != "second") {
        fprintf(stderr, "--wss must be first or second\n");
        return false;
      }
      o.p.wss = w == "second" ? 2 : 1;
    }
    else if (a == "-h" || a == "--help") {
      usage(argv[0]);
      exit(0);
    } else if (a.size() && a[0] != '-' && o.n_limit < 0) {
      o.n_limit = count("n_limit", a.c_str());  // gpu_svm4 positional form: ./gpu_svm4 <n_limit>
    } else {
      fprintf(stderr, "unknown argument %s\n", a.c_str());
      usage(argv[0]);
      return false;
    }
  }
  const svm_params& q = o.p;  // as SVMParams.__post_init__: a well-posed problem or an error
  if (!(q.C > 0) || !(q.gamma > 0) || !(q.tau > 0) || !(q.eps >= 0) || !(q.sv_tol >= 0) || q.max_iter < 1 ||
      !std::isfinite(q.C) || !std::isfinite(q.gamma) || !std::isfinite(q.tau)) {
    fprintf(stderr, "parameters out of range: C, gamma, tau > 0; eps, sv-tol >= 0; max-iter >= 1\n");
    return false;
  }
  if (o.train.empty()) o.train = o.dataset + "_train_data.csv";
  if (o.test.empty()) o.test = o.dataset + "_test_data.csv";
  return true;
}

struct Data {
  long long n = 0, d = 0;
  std::vector<double> X;
  std::vector<int32_t> y, raw;
};

// Train split: CSV (row-limited) or synthetic rows [0, N).  Test split: CSV or synthetic rows
// [N, N+M) of the same generator (disjoint samples, same distribution).
inline bool load_split(const Options& o, bool train, Data& out) {
  if (o.synth_train > 0) {
    long long n = train ? o.synth_train : o.synth_test;
    if (train && o.n_limit >= 0 && o.n_limit < n) n = o.n_limit;
    const long long off = train ? 0 : o.synth_train;
    out.n = n;
    out.d = 784;
    out.X.resize(size_t(n) * 784);
    out.raw.resize(size_t(n));
    if (svm_synth_mnist(o.seed, off, n, out.X.data(), out.raw.data(), 0) != SVM_OK) {
      fprintf(stderr, "%s\n", svm_last_error());
      return false;
    }
    out.y.resize(size_t(n));
    for (long long i = 0; i < n; ++i) out.y[size_t(i)] = out.raw[size_t(i)] == o.positive_label ? 1 : -1;
    return true;
  }
  const std::string& path = train ? o.train : o.test;
  const long long lim = train ? o.n_limit : o.test_limit;
  void* h = svm_csv_load(path.c_str(), lim, o.positive_label, 0);
  if (!h) {
    fprintf(stderr, "%s\n", svm_last_error());
    return false;
  }
  int64_t n, d;
  svm_dataset_dims(h, &n, &d);
  out.n = n;
  out.d = d;
  out.X.resize(size_t(n * d));
  out.y.resize(size_t(n));
  out.raw.resize(size_t(n));
  svm_dataset_copy(h, out.X.data(), out.y.data(), out.raw.data());
  svm_dataset_free(h);
  return true;
}

inline double ms_between(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

inline void write_json(const std::string& path, const char* program, const Options& o, long long n, long long d,
                       const svm_result& r, long long correct, long long m, double train_ms, double pred_ms,
                       double total_ms, const char* extra) {
  if (path.empty()) return;
  FILE* f = fopen(path.c_str(), "w");
  if (!f) {
    fprintf(stderr, "cannot write %s\n", path.c_str());
    return;
  }
  fprintf(f,
          "{\"program\": \"%s\", \"n\": %lld, \"n_features\": %lld, \"C\": %.17g, \"gamma\": %.17g, "
          "\"tau\": %.17g, \"iterations\": %lld, \"b\": %.17g, \"b_high\": %.17g, \"b_low\": %.17g, "
          "\"stop_reason\": \"%s\", \"n_sv\": %lld, \"test_correct\": %lld, \"test_m\": %lld, "
          "\"accuracy\": %.17g, \"training_ms\": %.3f, \"prediction_ms\": %.3f, \"total_ms\": %.3f%s%s}\n",
          program, n, d, o.p.C, o.p.gamma, o.p.tau, (long long)r.iterations, r.b, r.b_high, r.b_low,
          svm_stop_message(r.stop_reason), (long long)r.n_sv, correct, m, m ? double(correct) / double(m) : 0.0,
          train_ms, pred_ms, total_ms, extra && *extra ? ", " : "", extra ? extra : "");
  fclose(f);
}

}  // namespace cli
