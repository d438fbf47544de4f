// Distributed SMO over GPUs (dsmo.hip): types shared with the persistent solver core (persist.h).
//
// P teams of workgroups run ONE first-order SMO together.  Team t owns the contiguous training
// points [t * W, (t + 1) * W) (W = workgroups per team x points per workgroup) and the slab
// K(:, own) of the RBF Gram (n x W, exact-integer values); every iteration each workgroup publishes
// its candidate record into the receive array of EVERY team (its own GPU's and its peers', over
// xGMI) and sweeps its own team's array, so every workgroup of every GPU derives the same pair
// with the lowest-index rule and the trajectory is the single-GPU solve's, bit for bit.
#pragma once
#include <cstdint>

namespace svm355 {

constexpr int kMaxPeers = 8;  // teams of one distributed solve (one per GPU of a node)

// Receive arrays of the teams' exchange (device pointers valid on the launching GPU: its own array
// and its peers' arrays mapped over xGMI).  own = the team whose array a workgroup sweeps.
struct PeerExch {
  unsigned long long* arr[kMaxPeers];
  int n = 0;
  int own = 0;
};

// One team's slab: K(i, col0 + j) at slab[i * ldw + j], i < n, j < width.
struct DsmoTeam {
  const double* slab = nullptr;
  int64_t ldw = 0;
  int64_t col0 = 0;
};

// Self-validating record granule of the peer exchange: 32-bit payload, high word = epoch XOR an
// odd-multiplier mix of the payload (a bijection), so a granule whose halves come from different
// writes never validates for the epoch awaited unless it carries that epoch's payload (tearing of
// a 64-bit transfer over the fabric cannot produce a wrong value).
__host__ __device__ inline uint32_t peer_mix(uint32_t payload) { return payload * 0x9E3779B1u; }
__host__ __device__ inline unsigned long long peer_word(uint32_t epoch, uint32_t payload) {
  return (static_cast<unsigned long long>(epoch ^ peer_mix(payload)) << 32) | payload;
}
__host__ __device__ inline bool peer_valid(unsigned long long x, uint32_t epoch) {
  return static_cast<uint32_t>(x >> 32) == (epoch ^ peer_mix(static_cast<uint32_t>(x)));
}

}  // namespace svm355
