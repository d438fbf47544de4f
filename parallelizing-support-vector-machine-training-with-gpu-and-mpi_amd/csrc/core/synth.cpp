// Deterministic MNIST-shaped synthetic data (the reference's MNIST CSVs are not shipped with the
// reference repo).
//
// Shape and value domain match MNIST: 28x28 = 784 features, integer pixel intensities 0..255,
// mostly-zero background, labels 0..9 with the one-vs-rest target digit "1" (~11% of samples).
// Each class has a stroke skeleton (quadratic Bezier curves; class 1 is a near-vertical bar, class
// 0 a loop); every sample jitters the skeleton, applies a random affine map and stroke width, and
// is rasterised with anti-aliased distance-to-stroke shading plus sparse speckle noise. Classes
// overlap enough that an RBF SVM keeps a few percent of the samples as support vectors, as on
// MNIST. Sample i depends only on (seed, i), so any range can be generated independently and in
// parallel with identical results.
#include <cmath>
#include <cstring>

#include "internal.h"

using namespace svm355;

namespace {

constexpr int W = 28;
constexpr int D = W * W;
constexpr int kStyles = 6;
constexpr int kMaxCurves = 4;

inline uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  double uni() { return double(splitmix64(s) >> 11) * (1.0 / 9007199254740992.0); }
  double range(double a, double b) { return a + (b - a) * uni(); }
  int below(int n) { return int(uni() * n) % n; }
};

struct Curve {  // quadratic Bezier P0-P1-P2
  double x[3], y[3];
};

struct Glyph {
  int nc = 0;
  Curve c[kMaxCurves];
};

// Class skeletons in a 28x28 frame (x right, y down).
Glyph base_skeleton(int cls, Rng& r) {
  Glyph g;
  auto add = [&](double x0, double y0, double x1, double y1, double x2, double y2) {
    if (g.nc < kMaxCurves) g.c[g.nc++] = Curve{{x0, x1, x2}, {y0, y1, y2}};
  };
  switch (cls) {
    case 0:  // loop: two arcs
      add(14, 5, 4, 14, 14, 23);
      add(14, 23, 24, 14, 14, 5);
      break;
    case 1:  // bar with a slight slant
      add(15, 4, 14, 14, 13, 24);
      break;
    case 2:
      add(7, 9, 14, 1, 20, 9);
      add(20, 9, 14, 17, 7, 23);
      add(7, 23, 14, 23, 21, 23);
      break;
    case 3:
      add(7, 6, 19, 2, 15, 13);
      add(15, 13, 23, 20, 7, 22);
      break;
    case 4:
      add(17, 4, 9, 12, 6, 16);
      add(6, 16, 14, 16, 22, 16);
      add(17, 8, 17, 16, 17, 24);
      break;
    case 5:
      add(20, 5, 13, 5, 8, 5);
      add(8, 5, 7, 10, 9, 12);
      add(9, 12, 24, 15, 8, 23);
      break;
    case 6:
      add(17, 4, 6, 12, 9, 20);
      add(9, 20, 15, 27, 19, 18);
      add(19, 18, 13, 12, 9, 18);
      break;
    case 7:
      add(6, 6, 14, 6, 21, 6);
      add(21, 6, 16, 14, 12, 24);
      break;
    case 8:
      add(14, 4, 5, 9, 14, 14);
      add(14, 14, 23, 9, 14, 4);
      add(14, 14, 4, 19, 14, 24);
      add(14, 24, 24, 19, 14, 14);
      break;
    default:  // 9
      add(18, 9, 8, 2, 9, 11);
      add(9, 11, 16, 15, 18, 9);
      add(18, 9, 18, 16, 16, 24);
      break;
  }
  // Per-run variation of the skeleton itself (so the seed changes the problem, not just samples).
  for (int i = 0; i < g.nc; ++i)
    for (int k = 0; k < 3; ++k) {
      g.c[i].x[k] += r.range(-0.8, 0.8);
      g.c[i].y[k] += r.range(-0.8, 0.8);
    }
  return g;
}

void jitter(Glyph& g, Rng& r, double amt) {
  for (int i = 0; i < g.nc; ++i)
    for (int k = 0; k < 3; ++k) {
      g.c[i].x[k] += r.range(-amt, amt);
      g.c[i].y[k] += r.range(-amt, amt);
    }
}

inline double seg_dist2(double px, double py, double ax, double ay, double bx, double by) {
  const double vx = bx - ax, vy = by - ay, wx = px - ax, wy = py - ay;
  const double vv = vx * vx + vy * vy;
  double t = vv > 0 ? (wx * vx + wy * vy) / vv : 0.0;
  t = t < 0 ? 0 : (t > 1 ? 1 : t);
  const double dx = wx - t * vx, dy = wy - t * vy;
  return dx * dx + dy * dy;
}

void render(const Glyph& g, double thick, double ink, Rng& r, double* out) {
  constexpr int kSeg = 12;
  double sx[kMaxCurves][kSeg + 1], sy[kMaxCurves][kSeg + 1];
  double xmin = 1e9, xmax = -1e9, ymin = 1e9, ymax = -1e9;
  for (int c = 0; c < g.nc; ++c)
    for (int s = 0; s <= kSeg; ++s) {
      const double t = double(s) / kSeg, u = 1 - t;
      sx[c][s] = u * u * g.c[c].x[0] + 2 * u * t * g.c[c].x[1] + t * t * g.c[c].x[2];
      sy[c][s] = u * u * g.c[c].y[0] + 2 * u * t * g.c[c].y[1] + t * t * g.c[c].y[2];
      xmin = std::min(xmin, sx[c][s]);
      xmax = std::max(xmax, sx[c][s]);
      ymin = std::min(ymin, sy[c][s]);
      ymax = std::max(ymax, sy[c][s]);
    }
  const double half = 0.5 * thick;
  const double reach = half + 1.0;
  for (int py = 0; py < W; ++py)
    for (int px = 0; px < W; ++px) {
      const double cx = px + 0.5, cy = py + 0.5;
      double v = 0.0;
      if (cx >= xmin - reach && cx <= xmax + reach && cy >= ymin - reach && cy <= ymax + reach) {
        double best = 1e18;
        for (int c = 0; c < g.nc; ++c)
          for (int s = 0; s < kSeg; ++s)
            best = std::min(best, seg_dist2(cx, cy, sx[c][s], sy[c][s], sx[c][s + 1], sy[c][s + 1]));
        const double dist = std::sqrt(best);
        const double cover = std::min(1.0, std::max(0.0, half + 0.75 - dist));
        v = ink * cover;
      }
      // Sparse speckle (about 1.5% of pixels) so background columns are not all-constant.
      if (r.uni() < 0.015) v = std::max(v, r.range(10.0, 160.0));
      double q = std::floor(v + 0.5);
      if (q < 0) q = 0;
      if (q > 255) q = 255;
      out[py * W + px] = q;
    }
}

}  // namespace

extern "C" SVM_API int svm_synth_mnist(uint64_t seed, int64_t offset, int64_t n, double* X, int32_t* labels,
                                       int32_t n_threads) {
  if (n < 0 || offset < 0 || (n > 0 && (!X || !labels))) {
    set_error("svm_synth_mnist: bad arguments");
    return SVM_ERR_ARG;
  }
  // Class skeletons and per-class styles depend only on the seed.
  Glyph styles[10][kStyles];
  {
    uint64_t s = seed ^ 0xA5A5A5A5DEADBEEFull;
    Rng r(splitmix64(s));
    for (int c = 0; c < 10; ++c) {
      const Glyph base = base_skeleton(c, r);
      for (int k = 0; k < kStyles; ++k) {
        styles[c][k] = base;
        jitter(styles[c][k], r, 2.0);
      }
    }
  }
  // MNIST digit frequencies (train split), digit 1 ~ 11.2%.
  static const double freq[10] = {0.0987, 0.1124, 0.0993, 0.1022, 0.0974,
                                  0.0904, 0.0986, 0.1044, 0.0975, 0.0991};
  double cdf[10];
  double acc = 0;
  for (int c = 0; c < 10; ++c) cdf[c] = (acc += freq[c]);

  parallel_for(n, resolve_threads(n_threads), [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      const uint64_t gi = uint64_t(offset + i);  // global sample index
      uint64_t s = seed * 0x9E3779B97F4A7C15ull + gi * 0xD1B54A32D192ED03ull + 0x1234567ull;
      Rng r(splitmix64(s));
      const double u = r.uni() * acc;
      int cls = 0;
      while (cls < 9 && u > cdf[cls]) ++cls;
      Glyph g = styles[cls][r.below(kStyles)];
      jitter(g, r, 1.6);
      // Random affine about the centre: rotation, anisotropic scale, shear, shift.
      const double ang = r.range(-0.25, 0.25);
      const double scx = r.range(0.82, 1.15), scy = r.range(0.85, 1.12), sh = r.range(-0.2, 0.2);
      const double tx = r.range(-2.0, 2.0), ty = r.range(-2.0, 2.0);
      const double ca = std::cos(ang), sa = std::sin(ang);
      for (int c = 0; c < g.nc; ++c)
        for (int k = 0; k < 3; ++k) {
          const double x = g.c[c].x[k] - 14.0, y = g.c[c].y[k] - 14.0;
          const double x1 = scx * x + sh * y, y1 = scy * y;
          g.c[c].x[k] = 14.0 + ca * x1 - sa * y1 + tx;
          g.c[c].y[k] = 14.0 + sa * x1 + ca * y1 + ty;
        }
      const double thick = r.range(1.1, 3.0);
      const double ink = r.range(200.0, 255.0);
      render(g, thick, ink, r, X + i * D);
      labels[i] = cls;
    }
  });
  return SVM_OK;
}
