// Workgroup -> output-tile maps shared by the MFMA Gram kernels (gfx950, 8 XCDs).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace svm355 {

// Bijective remap: workgroups dispatched to the same XCD (orig % 8 under the round-robin dispatch
// of CDNA4) get a contiguous range of logical tile ids, so neighbouring tiles share an L2.  Speed
// only: correctness never depends on placement.
__device__ __forceinline__ int64_t xcd_remap(int64_t orig, int64_t nwg) {
  const int64_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// Upper-triangle tile enumeration: id -> (tm, tn) with tn >= tm, row-major (row tm holds T - tm
// tiles starting at offset(tm) = tm*T - tm*(tm-1)/2).
__device__ __forceinline__ void tri_tile(int64_t id, int64_t T, int64_t& tm, int64_t& tn) {
  const double b = double(2 * T + 1);
  int64_t r = int64_t((b - sqrt(b * b - 8.0 * double(id))) * 0.5);
  auto off = [T](int64_t x) { return x * T - x * (x - 1) / 2; };
  while (r > 0 && off(r) > id) --r;
  while (off(r + 1) <= id) ++r;
  tm = r;
  tn = r + (id - off(r));
}

}  // namespace svm355
