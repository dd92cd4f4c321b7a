// The loss's negatives, drawn and grouped by post in two levels (hgnn_draw_sort_negatives when
// the post ids fit 20 bits; the 3-pass LSD radix sort of csr_build.hip otherwise).
//
// What the fused dP gather needs (train_gnn.py:272-273's negatives, transposed): for every post,
// the users whose positive edge drew it, in position order — a stable sort of the E pairs
// (draw(i), a[i]) by draw.  The draws are counter-based (uniform_draw(seed, i, n_keys)), so any
// pass can recompute a key from its position instead of reading it.
//
//   level 1 (MSD bucket scatter): the top H bits of the key pick one of nb <= 1024 buckets.  A
//     count kernel histograms every 16384-item tile in LDS (keys drawn, nothing read); one scan
//     turns the (bucket, tile) counts into stable output offsets; the scatter kernel ranks its
//     tile by bucket in LDS (wave ballots + per-wave running counts), reorders it in LDS, and
//     writes each bucket's run contiguously: the key's low L bits (u16) and the payload a[i].
//     It also writes the draws in position order (the scoring pass's negatives).
//   level 2 (per-bucket counting sort): one workgroup per bucket, each wave a contiguous
//     sixteenth of it.  Per-wave LDS histograms of the low bits, one block scan (which is also
//     the bucket's slice of the post rowptr: no sorted keys are written, no binary search), then
//     each wave writes its payloads at per-key running offsets (k_negb_sort below).  Both levels
//     keep tile order and in-tile position order, so the sort is stable — bit-identical to the
//     LSD sort (GPU-tested).
//
// Measured at cfg4 (200M pairs, 2^20 posts): 5.5-5.9 ms against the LSD sort's 3.1 ms; an earlier
// level 2 that reordered 8192-item tiles in LDS took 1.43 ms for level 1 + 1.37 ms for level 2.
// Level 1's 1024-way scatter of 16384-item tiles leaves ~16 items per bucket per tile, so its
// writes are short runs, and both levels run one latency-bound block per CU in their LDS phases.
// Hence opt-in only (HGNN_NEG_SORT=2level; csr_build.hip).
//
// Bytes per pair: level 1 reads a[i] (4) and writes draw (4) + low key (2) + payload (4); level 2
// reads low key twice (2 + 2, the second mostly from the Infinity Cache) and the payload (4) and
// writes the payload (4): ~26 B against the LSD sort's ~60 B at cfg4 (3 passes of 8-B pairs plus
// their count passes).
#include "hgnn_common.h"

#include <stdlib.h>

namespace hgnn {

constexpr int kNbThreads = 1024;                  // 16 waves
constexpr int kNbWaves = kNbThreads / 64;
// level 1 tile: RR items per thread (16: 16384-item tiles, one block per CU; 8: 8192, two)
constexpr int kNbMaxDigits = 1024;                // H, L <= 10 bits

// Block-wide exclusive scan of one int per thread (1024 threads); returns the prefix.
__device__ __forceinline__ int nb_block_scan(int v, int* wsum /*[kNbWaves]*/) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int pre = 0;
#pragma unroll
  for (int q = 0; q < kNbWaves; ++q) pre += q < w ? wsum[q] : 0;
  __syncthreads();
  return pre + inc - v;
}

// Stable in-wave rank of `digit` among the wave's valid lanes (bits ballots), against the
// wave-private running count wcount[digit]; the first lane of each digit group bumps the count.
__device__ __forceinline__ int nb_wave_rank(int digit, bool valid, int bits, uint16_t* wcount) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  unsigned long long match = __ballot(valid);
  for (int b = 0; b < bits; ++b) {
    const unsigned long long m = __ballot((digit >> b) & 1);
    match &= ((digit >> b) & 1) ? m : ~m;
  }
  const int before = valid ? (int)wcount[digit] : 0;
  const int below = __popcll(match & lt);
  __builtin_amdgcn_wave_barrier();
  if (valid && below == 0) wcount[digit] = (uint16_t)(before + __popcll(match));
  __builtin_amdgcn_wave_barrier();
  return before + below;
}

// Tile-local digit starts and per-wave offsets from the per-wave counts (one digit per thread):
// wcount[w][d] becomes the tile offset of wave w's first item of digit d; returns d's tile total.
__device__ __forceinline__ int nb_tile_offsets(uint16_t (*wcount)[kNbMaxDigits], int* dstart,
                                               int* wsum) {
  const int d = threadIdx.x;
  int tot = 0;
#pragma unroll
  for (int w = 0; w < kNbWaves; ++w) tot += wcount[w][d];
  const int st = nb_block_scan(tot, wsum);
  dstart[d] = st;
  int o = st;
#pragma unroll
  for (int w = 0; w < kNbWaves; ++w) {
    const int c = wcount[w][d];
    wcount[w][d] = (uint16_t)o;
    o += c;
  }
  return tot;
}

__device__ __forceinline__ int64_t nb_xcd_tile(int64_t b, int64_t nb) {
  constexpr int kXcd = 8;    // hardware block b runs on XCD b % 8: give each XCD a tile range
  const int64_t q = nb / kXcd, r = nb % kXcd, x = b % kXcd, i = b / kXcd;
  return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// Level 1, count: counts[bucket * ntiles + tile] = #draws of the tile in the bucket.
template <int RR>
__global__ void __launch_bounds__(kNbThreads) k_negb_count(const uint64_t* d_seed, uint32_t hi,
                                                           int64_t E, int lbits, int nb,
                                                           int32_t* counts) {
  constexpr int kNbTile1 = kNbThreads * RR;
  __shared__ int hist[kNbMaxDigits];
  hist[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t seed = *d_seed;
  const int64_t tile = blockIdx.x, ntiles = gridDim.x;
  const int64_t base = tile * kNbTile1;
#pragma unroll 4
  for (int r = 0; r < RR; ++r) {
    const int64_t i = base + (int64_t)r * kNbThreads + threadIdx.x;
    if (i < E) atomicAdd(&hist[uniform_draw(seed, i, hi) >> lbits], 1);
  }
  __syncthreads();
  if ((int)threadIdx.x < nb) counts[(int64_t)threadIdx.x * ntiles + tile] = hist[threadIdx.x];
}

// Level 1, scatter: (low key, a[i]) of the tile to each bucket's run at offs[bucket, tile]; the
// draws to neg_out in position order.
template <int RR>
__global__ void __launch_bounds__(kNbThreads, RR <= 8 ? 8 : 4) k_negb_scatter(
    const uint64_t* __restrict__ d_seed, uint32_t hi, int64_t E, int hbits, int lbits, int nb,
    const int32_t* __restrict__ offs, const int32_t* __restrict__ a,
    int32_t* __restrict__ neg_out, uint16_t* __restrict__ keyl, int32_t* __restrict__ pay) {
  constexpr int kNbTile1 = kNbThreads * RR;
  constexpr int kNbRounds1 = RR;
  __shared__ uint16_t wcount[kNbWaves][kNbMaxDigits];   // 32 KB
  __shared__ uint16_t sidx[kNbTile1];                   // 32 / 16 KB: tile index, bucket order
  __shared__ int dstart[kNbMaxDigits];
  __shared__ int gbase[kNbMaxDigits];
  __shared__ int wsum[kNbWaves];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t ntiles = gridDim.x;
  const int64_t tile = nb_xcd_tile(blockIdx.x, ntiles);
  const int64_t tile0 = tile * kNbTile1;
#pragma unroll
  for (int q = 0; q < kNbWaves; ++q) wcount[q][threadIdx.x] = 0;
  if ((int)threadIdx.x < nb) gbase[threadIdx.x] = offs[(int64_t)threadIdx.x * ntiles + tile];
  __syncthreads();
  const uint64_t seed = *d_seed;
  const int64_t wave0 = tile0 + (int64_t)w * (kNbTile1 / kNbWaves);
  int packed[kNbRounds1];   // bucket | in-wave rank << 16, or -1
  // (the tile's payload lines are touched here so the write phase's gathers hit the cache)
  if (lane == 0 && wave0 < E) __builtin_prefetch(a + wave0, 0, 3);
#pragma unroll
  for (int r = 0; r < kNbRounds1; ++r) {
    const int64_t i = wave0 + r * 64 + lane;
    const bool valid = i < E;
    const int key = valid ? uniform_draw(seed, i, hi) : 0;
    if (valid && neg_out) neg_out[i] = key;
    const int digit = key >> lbits;
    const int rk = nb_wave_rank(digit, valid, hbits, wcount[w]);
    packed[r] = valid ? (digit | (rk << 16)) : -1;
  }
  __syncthreads();
  nb_tile_offsets(wcount, dstart, wsum);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kNbRounds1; ++r) {
    if (packed[r] >= 0) {
      const int digit = packed[r] & 0xFFFF;
      const int p = wcount[w][digit] + (packed[r] >> 16);
      sidx[p] = (uint16_t)(w * (kNbTile1 / kNbWaves) + r * 64 + lane);
    }
  }
  __syncthreads();
  // write phase, in bucket order: every payload gather (a[i], from the tile's 64 KB the ranking
  // just touched) issued before the stores
  const int n_tile = (int)min<int64_t>(kNbTile1, E - tile0);
  const int lmask = (1 << lbits) - 1;
  constexpr int HB = kNbRounds1 / 2;                   // two batches (register budget: 2 blocks/CU)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    int wpos[HB], vkey[HB], vpay[HB];
#pragma unroll
    for (int r = 0; r < HB; ++r) {
      const int j = (h * HB + r) * kNbThreads + threadIdx.x;
      wpos[r] = -1;
      if (j < n_tile) {
        const int64_t i = tile0 + sidx[j];
        const int key = uniform_draw(seed, i, hi);    // recomputed: cheaper than LDS space
        const int digit = key >> lbits;
        wpos[r] = gbase[digit] + (j - dstart[digit]);   // < E < 2^31
        vkey[r] = key & lmask;
        vpay[r] = a[i];
      }
    }
#pragma unroll
    for (int r = 0; r < HB; ++r) {
      if (wpos[r] >= 0) {
        keyl[wpos[r]] = (uint16_t)vkey[r];
        pay[wpos[r]] = vpay[r];
      }
    }
  }
}

// Level 2: bucket b = blockIdx.x, items [offs[b, 0], offs[b + 1, 0]).  Each wave takes a
// contiguous sixteenth of the bucket: it histograms its low keys into its own LDS row; one block
// scan over (key, wave) turns the rows into each wave's start offset per key (and the bucket's
// slice of rowptr); then every wave walks its range in rounds of 64 and writes each payload at
// its key's running offset — wave ballots rank equal keys within a round, the wave's running
// counters carry the order across rounds, so the result is stable with no block barrier per
// round.  The bucket's output (~0.8 MB at cfg4) is written in place of an LDS reorder: its lines
// merge in the caches.
constexpr int kNbPrefetch = 8;                        // rounds of loads in flight per wave

__global__ void __launch_bounds__(kNbThreads) k_negb_sort(
    const int32_t* __restrict__ offs, int64_t ntiles, int nb, int64_t E, int64_t n_keys,
    int lbits, const uint16_t* __restrict__ keyl, const int32_t* __restrict__ pay,
    int32_t* __restrict__ rowptr, int32_t* __restrict__ out) {
  __shared__ int wcnt[kNbWaves][kNbMaxDigits];          // 64 KB
  __shared__ int wsum[kNbWaves];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, d = threadIdx.x;
  const int b = blockIdx.x;
  const int64_t bs = offs[(int64_t)b * ntiles];
  const int64_t be = b + 1 < nb ? (int64_t)offs[(int64_t)(b + 1) * ntiles] : E;
  const int R = 1 << lbits;
  const int64_t per = ((be - bs + kNbWaves - 1) / kNbWaves + 63) / 64 * 64;
  const int64_t w0 = min<int64_t>(bs + (int64_t)w * per, be);
  const int64_t w1 = min<int64_t>(w0 + per, be);
#pragma unroll
  for (int q = 0; q < kNbWaves; ++q) wcnt[q][d] = 0;
  __syncthreads();
  // per-wave histogram: 16 loads in flight per lane per batch
  for (int64_t k0 = w0; k0 < w1; k0 += 16 * 64) {
    int kk[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t k = k0 + q * 64 + lane;
      kk[q] = k < w1 ? (int)keyl[k] : -1;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (kk[q] >= 0) atomicAdd(&wcnt[w][kk[q]], 1);
  }
  __syncthreads();
  // key d: total over the waves, bucket-wide start (scan over keys), per-wave starts
  int tot = 0;
#pragma unroll
  for (int q = 0; q < kNbWaves; ++q) tot += wcnt[q][d];
  const int st = nb_block_scan(d < R ? tot : 0, wsum);
  const int64_t key = ((int64_t)b << lbits) + d;
  if (d < R && key < n_keys) rowptr[key] = (int32_t)(bs + st);
  if (b == nb - 1 && d == 0) rowptr[n_keys] = (int32_t)E;
  {
    int o = (int)bs + st;
#pragma unroll
    for (int q = 0; q < kNbWaves; ++q) {
      const int c = wcnt[q][d];
      wcnt[q][d] = o;
      o += c;
    }
  }
  __syncthreads();
  // per-wave stable scatter; loads kNbPrefetch rounds ahead
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int* cnt = wcnt[w];
  int ql[kNbPrefetch], qu[kNbPrefetch];
#pragma unroll
  for (int r = 0; r < kNbPrefetch; ++r) {
    const int64_t k = w0 + r * 64 + lane;
    ql[r] = k < w1 ? (int)keyl[k] : -1;
    qu[r] = k < w1 ? pay[k] : 0;
  }
  for (int64_t k0 = w0; k0 < w1; k0 += kNbPrefetch * 64) {
#pragma unroll
    for (int r = 0; r < kNbPrefetch; ++r) {
      const int l = ql[r], u = qu[r];
      const int64_t kn = k0 + (r + kNbPrefetch) * 64 + lane;    // refill this slot
      ql[r] = kn < w1 ? (int)keyl[kn] : -1;
      qu[r] = kn < w1 ? pay[kn] : 0;
      const bool valid = l >= 0;
      unsigned long long match = __ballot(valid);
      if (match == 0) continue;
      for (int bb = 0; bb < lbits; ++bb) {
        const unsigned long long m = __ballot((l >> bb) & 1);
        match &= ((l >> bb) & 1) ? m : ~m;
      }
      const int before = valid ? cnt[l] : 0;
      const int below = __popcll(match & lt);
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) cnt[l] = before + __popcll(match);
      __builtin_amdgcn_wave_barrier();
      if (valid) out[before + below] = u;
    }
  }
}

bool negatives_two_level_applies(int64_t E, int64_t n_keys) {
  return E > 0 && n_keys >= 1 && n_keys <= (int64_t(1) << 20) && E < (int64_t(1) << 31) - 1;
}

size_t negatives_two_level_ws_bytes(int64_t E, int64_t n_keys) {
  int bits = 0;
  while ((int64_t(1) << bits) < n_keys) ++bits;
  const int hbits = bits < 10 ? bits : 10;
  const int lbits = bits - hbits;
  const int64_t nb = ((n_keys - 1) >> lbits) + 1;
  const int64_t ntiles = cdiv(E, kNbThreads * 8);   // the larger count of both tile sizes
  size_t scan_b = 0;
  exclusive_scan_i32(nullptr, nullptr, nb * ntiles, nullptr, &scan_b, 0);
  return align_up((size_t)E * 2, 256) + align_up((size_t)E * 4, 256) +
         2 * align_up((size_t)(nb * ntiles + 1) * 4, 256) + scan_b + 1024;
}

int negatives_two_level(const uint64_t* d_seed, const int32_t* a, int64_t E, int64_t n_keys,
                        int32_t* neg_out, int32_t* rowptr, int32_t* a_sorted, void* ws,
                        size_t ws_bytes, hipStream_t stream) {
  int bits = 0;
  while ((int64_t(1) << bits) < n_keys) ++bits;   // keys in [0, n_keys)
  const int hbits = bits < 10 ? bits : 10;        // <= 1024 buckets, ...
  const int lbits = bits - hbits;                 // ... each <= 1024 keys wide
  const int nb = (int)(((n_keys - 1) >> lbits) + 1);
  static const int rr = getenv("HGNN_NEGB_ROUNDS") ? atoi(getenv("HGNN_NEGB_ROUNDS")) : 16;
  const int64_t ntiles = cdiv(E, (int64_t)kNbThreads * (rr == 8 ? 8 : 16));
  if (ws_bytes < negatives_two_level_ws_bytes(E, n_keys))
    return fail(HGNN_E_WS, "draw_sort_negatives: workspace too small");
  Workspace w(ws, ws_bytes);
  uint16_t* keyl = w.take<uint16_t>(E);
  int32_t* pay = w.take<int32_t>(E);
  int32_t* counts = w.take<int32_t>(nb * ntiles + 1);
  int32_t* offs = w.take<int32_t>(nb * ntiles + 1);
  size_t scan_b = 0;
  exclusive_scan_i32(nullptr, nullptr, nb * ntiles, nullptr, &scan_b, stream);
  void* scan_ws = w.take<char>(scan_b);
  if (!scan_ws) return fail(HGNN_E_WS, "draw_sort_negatives: workspace too small");
  const uint32_t hi = (uint32_t)n_keys;
  if (rr == 8)
    hipLaunchKernelGGL(k_negb_count<8>, dim3((unsigned)ntiles), dim3(kNbThreads), 0, stream,
                       d_seed, hi, E, lbits, nb, counts);
  else
    hipLaunchKernelGGL(k_negb_count<16>, dim3((unsigned)ntiles), dim3(kNbThreads), 0, stream,
                       d_seed, hi, E, lbits, nb, counts);
  if (int rc = check_launch("k_negb_count")) return rc;
  if (int rc = exclusive_scan_i32(counts, offs, nb * ntiles, scan_ws, &scan_b, stream)) return rc;
  if (rr == 8)
    hipLaunchKernelGGL(k_negb_scatter<8>, dim3((unsigned)ntiles), dim3(kNbThreads), 0, stream,
                       d_seed, hi, E, hbits, lbits, nb, (const int32_t*)offs, a, neg_out, keyl,
                       pay);
  else
    hipLaunchKernelGGL(k_negb_scatter<16>, dim3((unsigned)ntiles), dim3(kNbThreads), 0, stream,
                       d_seed, hi, E, hbits, lbits, nb, (const int32_t*)offs, a, neg_out, keyl,
                       pay);
  if (int rc = check_launch("k_negb_scatter")) return rc;
  hipLaunchKernelGGL(k_negb_sort, dim3((unsigned)nb), dim3(kNbThreads), 0, stream,
                     (const int32_t*)offs, ntiles, nb, E, n_keys, lbits, (const uint16_t*)keyl,
                     (const int32_t*)pay, rowptr, a_sorted);
  return check_launch("k_negb_sort");
}

}  // namespace hgnn
