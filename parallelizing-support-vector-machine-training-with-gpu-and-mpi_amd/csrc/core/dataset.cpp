// L0 data I/O: CSV loader/writer.
//
// Semantics follow read_CSV (main3.cpp:13-54; row-limited variant gpu_svm_main4.cu:16-59):
//   * the first line is a header; n_features = (#header fields) - 1, the last column is the label;
//   * data lines with < 2 fields are skipped;
//   * every feature cell is parsed as a double, the label as an integer;
//   * y = +1 iff label == positive_label (reference: positive_label = 1), else -1;
//   * with a row limit, the counter includes skipped lines (gpu_svm_main4.cu:34-38).
// Unlike the reference's per-cell std::stringstream parse, the file is read once into memory,
// split into lines, and parsed in parallel with std::from_chars (same values as std::stod for
// decimal input).
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <vector>

#include "internal.h"

namespace svm355 {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

namespace {

struct Dataset {
  int64_t n = 0, d = 0;
  std::vector<double> X;
  std::vector<int32_t> y, raw;
};

// Split [s, e) on ',' into field spans; returns field count.
inline size_t split_fields(const char* s, const char* e, std::vector<std::pair<const char*, const char*>>& out) {
  out.clear();
  const char* p = s;
  // std::getline(ss, cell, ',') semantics: a trailing empty field after the last comma is dropped.
  while (p < e) {
    const char* q = static_cast<const char*>(memchr(p, ',', size_t(e - p)));
    if (!q) {
      out.emplace_back(p, e);
      break;
    }
    out.emplace_back(p, q);
    p = q + 1;
  }
  return out.size();
}

inline const char* skip_ws(const char* p, const char* e) {
  while (p < e && (*p == ' ' || *p == '\t')) ++p;
  return p;
}

bool parse_double(const char* s, const char* e, double& v) {
  s = skip_ws(s, e);
  if (s < e && *s == '+') ++s;
  auto r = std::from_chars(s, e, v);
  return r.ec == std::errc() && std::isfinite(v);  // "nan" / "inf" cells: rejected, not trained on
}

bool parse_int(const char* s, const char* e, int32_t& v) {
  s = skip_ws(s, e);
  if (s < e && *s == '+') ++s;
  auto r = std::from_chars(s, e, v);
  if (r.ec == std::errc()) return true;
  // std::stoi accepts "1.0"-style labels by truncation; emulate via double parse.
  double dv;
  if (parse_double(s, e, dv)) {
    v = int32_t(dv);
    return true;
  }
  return false;
}

}  // namespace
}  // namespace svm355

using namespace svm355;

extern "C" {

SVM_API const char* svm_last_error(void) { return g_last_error.c_str(); }

SVM_API void svm_default_params(svm_params* p) {
  if (!p) return;
  p->C = 10.0;
  p->gamma = 0.00125;
  p->tau = 1e-5;
  p->eps = 1e-12;
  p->sv_tol = 1e-8;
  p->max_iter = 100000;
  p->n_threads = 1;
  p->verbose = 0;
  p->wss = 1;
  p->shrink = 0;
}

SVM_API const char* svm_stop_message(int32_t reason) {
  switch (reason) {
    case SVM_STOP_CONVERGED: return "converged";
    case SVM_STOP_NO_CANDIDATE: return "i_high or i_low not found; iteration stops";
    case SVM_STOP_INFEASIBLE: return "warning: infeasible U and V; iteration stops";
    case SVM_STOP_NONPOS_ETA: return "warning: non positive eta; iteration stops";
    case SVM_STOP_MAX_ITER: return "Too many iterations; stopping";
    default: return "running";
  }
}

SVM_API void* svm_csv_load(const char* path, int64_t limit, int32_t positive_label, int32_t n_threads) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f.is_open()) {
    set_error("Error opening file: %s", path);
    return nullptr;
  }
  const std::streamsize size = f.tellg();
  f.seekg(0);
  std::string buf(size_t(size), '\0');
  if (size > 0 && !f.read(&buf[0], size)) {
    set_error("Error reading file: %s", path);
    return nullptr;
  }
  const char* b = buf.data();
  const char* e = b + buf.size();

  // Line spans (strip '\r' for CRLF files).
  std::vector<std::pair<const char*, const char*>> lines;
  lines.reserve(size_t(size / 1024 + 16));
  for (const char* p = b; p < e;) {
    const char* q = static_cast<const char*>(memchr(p, '\n', size_t(e - p)));
    const char* le = q ? q : e;
    const char* lr = (le > p && le[-1] == '\r') ? le - 1 : le;
    lines.emplace_back(p, lr);
    if (!q) break;
    p = q + 1;
  }
  if (lines.empty()) {
    set_error("Error: No data read from file.");
    return nullptr;
  }
  std::vector<std::pair<const char*, const char*>> fields;
  const int64_t n_header = int64_t(split_fields(lines[0].first, lines[0].second, fields));
  if (n_header < 2) {
    set_error("Error: header of %s has fewer than 2 columns", path);
    return nullptr;
  }
  auto ds = std::make_unique<Dataset>();
  ds->d = n_header - 1;

  // Data lines considered: the reference's G4 counter k counts every line read, kept or not.
  int64_t n_lines = int64_t(lines.size()) - 1;
  if (limit >= 0 && limit < n_lines) n_lines = limit;
  // A trailing empty line produced by a final '\n' is a skipped (short) line, as in getline.

  // Pass 1 (parallel): classify lines as kept (>= 2 fields) and validate the column count.
  std::vector<uint8_t> keep(size_t(std::max<int64_t>(n_lines, 0)), 0);
  const int32_t nt = resolve_threads(n_threads);
  parallel_for(n_lines, nt, [&](int64_t lo, int64_t hi) {
    std::vector<std::pair<const char*, const char*>> fl;
    for (int64_t i = lo; i < hi; ++i) {
      const auto& L = lines[size_t(i + 1)];
      const size_t nf = split_fields(L.first, L.second, fl);
      keep[size_t(i)] = nf >= 2;
    }
  });
  std::vector<int64_t> row_of(keep.size(), -1);
  int64_t n = 0;
  for (size_t i = 0; i < keep.size(); ++i)
    if (keep[i]) row_of[i] = n++;
  if (n == 0) {
    set_error("Error: No data read from file.");
    return nullptr;
  }
  ds->n = n;
  ds->X.assign(size_t(n * ds->d), 0.0);
  ds->y.assign(size_t(n), -1);
  ds->raw.assign(size_t(n), 0);

  const int64_t d = ds->d;
  // Pass 2 (parallel): parse.  Split evenly by line index with deterministic output placement.
  std::vector<int64_t> err_line(size_t(nt), -1);
  {
    const int64_t chunk = (n_lines + nt - 1) / nt;
    std::vector<std::thread> pool;
    for (int32_t w = 0; w < nt; ++w) {
      const int64_t lo = int64_t(w) * chunk, hi = std::min(n_lines, lo + chunk);
      if (lo >= hi) continue;
      pool.emplace_back([&, w, lo, hi] {
        std::vector<std::pair<const char*, const char*>> fl;
        for (int64_t i = lo; i < hi; ++i) {
          if (!keep[size_t(i)]) continue;
          const auto& L = lines[size_t(i + 1)];
          const size_t nf = split_fields(L.first, L.second, fl);
          const int64_t r = row_of[size_t(i)];
          double* xr = ds->X.data() + r * d;
          // Reference pushes nf-1 features per line; rows of other widths would misalign the
          // flat array, so we require exactly d features and report the offending line.
          if (int64_t(nf) - 1 != d) {
            err_line[size_t(w)] = i + 2;
            return;
          }
          for (int64_t k = 0; k < d; ++k) {
            if (!parse_double(fl[size_t(k)].first, fl[size_t(k)].second, xr[k])) {
              err_line[size_t(w)] = i + 2;
              return;
            }
          }
          int32_t lab;
          if (!parse_int(fl.back().first, fl.back().second, lab)) {
            err_line[size_t(w)] = i + 2;
            return;
          }
          ds->raw[size_t(r)] = lab;
          ds->y[size_t(r)] = (lab == positive_label) ? 1 : -1;
        }
      });
    }
    for (auto& th : pool) th.join();
  }
  for (int32_t w = 0; w < nt; ++w) {
    if (err_line[size_t(w)] >= 0) {
      set_error("Error: malformed CSV line %lld in %s (expected %lld finite features + label)",
                (long long)err_line[size_t(w)], path, (long long)d);
      return nullptr;
    }
  }
  return ds.release();
}

SVM_API int svm_dataset_dims(void* h, int64_t* n, int64_t* d) {
  if (!h) {
    set_error("null dataset handle");
    return SVM_ERR_ARG;
  }
  auto* ds = static_cast<Dataset*>(h);
  if (n) *n = ds->n;
  if (d) *d = ds->d;
  return SVM_OK;
}

SVM_API int svm_dataset_copy(void* h, double* X, int32_t* y, int32_t* raw_labels) {
  if (!h) {
    set_error("null dataset handle");
    return SVM_ERR_ARG;
  }
  auto* ds = static_cast<Dataset*>(h);
  if (X) memcpy(X, ds->X.data(), ds->X.size() * sizeof(double));
  if (y) memcpy(y, ds->y.data(), ds->y.size() * sizeof(int32_t));
  if (raw_labels) memcpy(raw_labels, ds->raw.data(), ds->raw.size() * sizeof(int32_t));
  return SVM_OK;
}

SVM_API void svm_dataset_free(void* h) { delete static_cast<Dataset*>(h); }

SVM_API int svm_csv_write(const char* path, const double* X, const int32_t* labels, int64_t n, int64_t d) {
  FILE* fp = fopen(path, "wb");
  if (!fp) {
    set_error("Error opening file for writing: %s", path);
    return SVM_ERR_IO;
  }
  std::string line;
  line.reserve(size_t(d) * 8 + 16);
  for (int64_t k = 0; k < d; ++k) {
    line += "f" + std::to_string(k) + ",";
  }
  line += "label\n";
  fwrite(line.data(), 1, line.size(), fp);
  char num[64];
  for (int64_t i = 0; i < n; ++i) {
    line.clear();
    for (int64_t k = 0; k < d; ++k) {
      const double v = X[i * d + k];
      // Integers print exactly; other values round-trip with %.17g.
      if (v == double(int64_t(v)) && v > -1e15 && v < 1e15)
        snprintf(num, sizeof(num), "%lld,", (long long)v);
      else
        snprintf(num, sizeof(num), "%.17g,", v);
      line += num;
    }
    snprintf(num, sizeof(num), "%d\n", labels[i]);
    line += num;
    if (fwrite(line.data(), 1, line.size(), fp) != line.size()) {
      fclose(fp);
      set_error("Error writing %s", path);
      return SVM_ERR_IO;
    }
  }
  fclose(fp);
  return SVM_OK;
}

}  // extern "C"
