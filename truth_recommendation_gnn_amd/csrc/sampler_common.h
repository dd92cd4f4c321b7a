// Device helpers shared by the eager sampler (sampler.hip) and the sync-free static one
// (sampler_static.hip): the counter-based draws, one destination's sample, the relabel hash set.
#pragma once
#include "hgnn_common.h"

namespace hgnn {

constexpr int kHopMax = 8;   // relations per hop (hgnn_sample_hop_*)

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// uniform integer in [0, m) from the draw (seed, node, r); Lemire's multiply-shift
__device__ __forceinline__ uint32_t draw(uint64_t seed, int32_t node, int r, uint32_t m) {
  const uint64_t h = splitmix64(seed * 0xD1B54A32D192ED03ull + ((uint64_t)(uint32_t)node << 8) +
                                (uint64_t)r);
  return (uint32_t)(((h >> 32) * (uint64_t)m) >> 32);
}

// A destination id outside [0, n_rows) has no neighbours (count 0): the caller validates the ids
// it was given with the first read-back it makes anyway, and nothing is read out of bounds.
__device__ __forceinline__ int32_t sample_count(const int32_t* rowptr, int64_t n_rows, int32_t d,
                                                int32_t fanout) {
  if (d < 0 || d >= n_rows) return 0;
  const int32_t deg = rowptr[d + 1] - rowptr[d];
  return (fanout < 0 || deg <= fanout) ? deg : fanout;
}

// G lanes (64: a wave; 16: a quarter wave, fanout <= 16) sample destination d into out[0 ..
// count).  Floyd: for jj = deg-k .. deg-1 draw t in [0, jj]; take t unless already taken, then jj;
// the chosen positions are held one per lane of the group, "already taken?" is one ballot masked
// to the group.  The draws and choices do not depend on G (a quarter wave samples what a wave
// does); fanout is one per launch, so every group still sampling runs the same iterations.
template <int G>
__device__ __forceinline__ void sample_fill(const int32_t* rowptr, const int32_t* col,
                                            int64_t n_rows, int32_t d, int32_t fanout,
                                            uint64_t seed, int32_t* out) {
  const int lane = threadIdx.x & 63;
  const int gl = lane % G;
  if (d < 0 || d >= n_rows) return;   // counted 0
  const int32_t beg = rowptr[d], deg = rowptr[d + 1] - beg;
  if (fanout < 0 || deg <= fanout) {   // keep every neighbour, in CSR order
    for (int32_t j = gl; j < deg; j += G) out[j] = col[beg + j];
    return;
  }
  int32_t chosen = -1;
  for (int r = 0; r < fanout; ++r) {
    const int32_t jj = deg - fanout + r;
    const int32_t t = (int32_t)draw(seed, d, r, (uint32_t)jj + 1u);
    const uint64_t bal = __ballot(gl < r && chosen == t);
    const bool taken = G == 64 ? bal != 0ull
                               : ((bal >> ((lane / G) * G)) & ((1ull << G) - 1ull)) != 0ull;
    if (gl == r) chosen = taken ? jj : t;
  }
  if (gl < fanout) out[gl] = col[beg + chosen];
}

// slot of `key` in an open-addressing table (key[] -1 = empty, capacity mask + 1, a power of two,
// at least twice the keys inserted); *found = the key was already there (inserted by another
// thread)
__device__ __forceinline__ uint32_t rl_find_or_insert(int32_t* keys, uint32_t mask, int shift,
                                                      int32_t key, bool* found = nullptr) {
  uint32_t s = (uint32_t)(((uint64_t)(uint32_t)key * 0x9E3779B97F4A7C15ull) >> shift);
  for (uint32_t probe = 0; probe <= mask; ++probe) {   // ends: load factor <= 1/2
    const int32_t k = __atomic_load_n(&keys[s], __ATOMIC_RELAXED);
    if (k == key) {
      if (found) *found = true;
      return s;
    }
    if (k == -1) {
      const int32_t old = atomicCAS(&keys[s], -1, key);
      if (old == -1) return s;
      if (old == key) {
        if (found) *found = true;
        return s;
      }
    }
    s = (s + 1) & mask;
  }
  return 0;   // unreachable with the capacity the host sizes
}

inline int64_t relabel_cap(int64_t n) {
  int64_t c = 64;
  while (c < 2 * n) c <<= 1;
  return c;
}

}  // namespace hgnn
