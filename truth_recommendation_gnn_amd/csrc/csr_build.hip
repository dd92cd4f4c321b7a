// K5: COO -> CSR by a stable LSD radix sort (8-bit digits), the device scan it needs, and the
// degree-skew plan.  Integer work, HBM/latency bound; no MFMA.
//
// Why a sort and not an atomic counting fill: the fill would order each row's edges by atomic
// arrival, so the fp32 sum order — and the last bits of every aggregate — would change from run
// to run.  A stable sort keeps each row in COO order (the order PyG scatters in), which makes the
// whole forward/backward bitwise reproducible and lets tests compare the CSR bit for bit with
// oracle/csr_ref.py.
#include "hgnn_common.h"

#include <stdlib.h>

namespace hgnn {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ------------------------------------------------------------------------------------------
// Exclusive scan (int32), three phases: tile sums -> scan of tile sums (recursive) -> tile scan.
// ------------------------------------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;                        // per thread
constexpr int kScanTile = kScanThreads * kScanItems;  // 4096

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Block-wide exclusive scan of one value per thread; returns the block total in *total.
__device__ __forceinline__ int block_excl_scan(int v, int* lds /*[kScanThreads/64]*/, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = wave_incl_scan(v);
  if (lane == 63) lds[wid] = inc;
  __syncthreads();
  int wpre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / 64; ++w) {
    int s = lds[w];
    wpre += (w < wid) ? s : 0;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return wpre + inc - v;
}

__global__ void __launch_bounds__(kScanThreads) k_tile_sums(const int32_t* in, int64_t n,
                                                            int32_t* sums) {
  __shared__ int lds[kScanThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  int s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    int64_t idx = base + (int64_t)i * kScanThreads + threadIdx.x;
    s += idx < n ? in[idx] : 0;
  }
  int tot;
  block_excl_scan(s, lds, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// out[i] = offs[tile] + exclusive prefix of in within the tile; out[n] = grand total when the
// last tile writes it (total pointer).
__global__ void __launch_bounds__(kScanThreads) k_tile_scan(const int32_t* in, int64_t n,
                                                            const int32_t* offs, int32_t* out,
                                                            int write_total) {
  __shared__ int lds[kScanThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int v[kScanItems];
  int s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    int64_t idx = base + i;
    v[i] = idx < n ? in[idx] : 0;
    s += v[i];
  }
  int tot;
  int pre = block_excl_scan(s, lds, &tot) + (offs ? offs[blockIdx.x] : 0);
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    int64_t idx = base + i;
    if (idx < n) out[idx] = pre;
    pre += v[i];
  }
  if (write_total && blockIdx.x == gridDim.x - 1 && threadIdx.x == kScanThreads - 1) out[n] = pre;
}

static size_t scan_ws_bytes(int64_t n) {
  size_t b = 0;
  while (n > kScanTile) {
    int64_t t = cdiv(n, kScanTile);
    b += align_up((size_t)(t + 1) * 4, 256);
    n = t;
  }
  return b + 256;
}

// Recursive: ws holds the tile-sum levels.
int exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t* ws_bytes,
                       hipStream_t stream) {
  if (!ws) {
    *ws_bytes = scan_ws_bytes(n);
    return HGNN_OK;
  }
  if (n <= 0) {
    (void)hipMemsetAsync(out, 0, sizeof(int32_t), stream);
    return check_launch("scan(empty)");
  }
  int64_t tiles = cdiv(n, kScanTile);
  if (tiles == 1) {
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(kScanThreads), 0, stream, in, n,
                       (const int32_t*)nullptr, out, 1);
    return check_launch("k_tile_scan");
  }
  Workspace w(ws, *ws_bytes);
  int32_t* sums = w.take<int32_t>(tiles + 1);
  size_t rest = w.cap > w.used ? w.cap - align_up(w.used, 256) : 0;
  void* rest_p = w.base + align_up(w.used, 256);
  if (!sums) return fail(HGNN_E_WS, "scan workspace too small");
  hipLaunchKernelGGL(k_tile_sums, dim3(tiles), dim3(kScanThreads), 0, stream, in, n, sums);
  if (int rc = check_launch("k_tile_sums")) return rc;
  if (int rc = exclusive_scan_i32(sums, sums, tiles, rest_p, &rest, stream)) return rc;
  hipLaunchKernelGGL(k_tile_scan, dim3(tiles), dim3(kScanThreads), 0, stream, in, n,
                     (const int32_t*)sums, out, 1);
  return check_launch("k_tile_scan");
}

// In-place use above (sums -> sums) is safe: k_tile_scan with a single tile reads all inputs into
// registers before writing; with several tiles each block reads/writes only its own tile after
// the tile sums were taken into a separate level.  (The nested call scans `sums` in place only
// when it fits one tile, or recursively with its own level.)

// ------------------------------------------------------------------------------------------
// Stable LSD radix sort of (key32, idx32) pairs, 8-bit digits.
// ------------------------------------------------------------------------------------------
// 8192-item tiles (512 threads x 16 rounds; round 4): per 7-bit digit a tile writes runs of ~64
// items instead of ~32.  A/B on the cfg4 negatives (200M draws over 1M posts, scripts/
// gpu_sort_ab.sh): 3.03 ms at 256 x 16, 3.42 at 256 x 32, 2.87 at 512 x 16; two passes of
// 10-bit digits (32 B per pair moved instead of ~52) measured 4.1-4.7 ms at every tile size —
// the ranking's ballots and the 1024-digit tables cost more than the third pass's bytes.
#ifndef HGNN_SORT_THREADS
#define HGNN_SORT_THREADS 512
#endif
#ifndef HGNN_SORT_ROUNDS
#define HGNN_SORT_ROUNDS 16
#endif
constexpr int kSortThreads = HGNN_SORT_THREADS;
constexpr int kSortRounds = HGNN_SORT_ROUNDS;             // one item per thread per round
constexpr int kSortTile = kSortThreads * kSortRounds;     // 8192 items per block
constexpr int kMaxRadix = 1024;

// key32 = key if both endpoints valid, else n_keys (sentinel sorts last); counts invalid edges.
__global__ void __launch_bounds__(256) k_prepare_keys(const int64_t* key, const int64_t* other,
                                                      int64_t E, int64_t n_keys, int64_t n_other,
                                                      int32_t* key32, int32_t* invalid) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int bad = 0;
  if (i < E) {
    int64_t k = key[i], o = other[i];
    bool ok = k >= 0 && k < n_keys && o >= 0 && o < n_other;
    key32[i] = ok ? (int32_t)k : (int32_t)n_keys;
    bad = ok ? 0 : 1;
  }
  unsigned long long m = __ballot(bad);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(invalid, __popcll(m));
}

// counts[digit * nblocks + block] for this block's tile (RADIX = 1 << BITS digits).  Every key of
// the tile is loaded before the first LDS atomic, so all RR loads per thread are in flight.
// GEN: the keys are the uniform draws uniform_draw(*gen.seed, i, gen.hi) (the negatives sort),
// computed in place of the key load.
struct KeyGen {
  const uint64_t* seed;
  uint32_t hi;
};

__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t nb);

// One LDS counter per digit.  (Measured and not kept, round 5: one counter per (digit, lane
// mod 32), conflict-free — count conflicts 4.7 -> 0 per LDS instruction, the cfg4 draw + sort
// 2.862 -> 2.888 ms; the conflicts are ~1 % of the kernel's wave-cycles)
template <int BITS, int RR = kSortRounds, bool GEN = false>
__global__ void __launch_bounds__(kSortThreads) k_digit_counts(const int32_t* keys, int64_t E,
                                                               int shift, int32_t* counts,
                                                               KeyGen gen = KeyGen{nullptr, 0}) {
  constexpr int R = 1 << BITS;
  __shared__ int hist[R];
  for (int dd = threadIdx.x; dd < R; dd += kSortThreads) hist[dd] = 0;
  // XCD-aware tile order as in k_digit_scatter: neighbouring tiles' count words (one line holds
  // 16 tiles' counts of a digit) are written from one XCD's L2 instead of eight
  const int64_t tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t base = tile * (kSortThreads * RR);
  int k[RR];
  const uint64_t seed = GEN ? *gen.seed : 0;
#pragma unroll
  for (int r = 0; r < RR; ++r) {
    const int64_t i = base + (int64_t)r * kSortThreads + threadIdx.x;
    k[r] = i < E ? (GEN ? uniform_draw(seed, i, gen.hi) : keys[i]) : -1;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RR; ++r)
    if (k[r] >= 0) atomicAdd(&hist[(k[r] >> shift) & (R - 1)], 1);
  __syncthreads();
  for (int dd = threadIdx.x; dd < R; dd += kSortThreads)
    counts[(int64_t)dd * gridDim.x + tile] = hist[dd];
}

// Stable scatter, block-local sort first.  Tile = kSortTile items; wave w owns the contiguous
// items [w*1024, (w+1)*1024) and walks them in 16 rounds of 64, ranking each item among equal
// digits with BITS ballots and a wave-private running count in LDS (no block barrier per round).
// The tile is then reordered by (digit, original index) in LDS and written out in per-digit
// runs, so global stores are contiguous runs instead of scattered words.  Carries up to two
// 32-bit payloads (a: identity when identity_a is set; b optional).
// XCD-aware tile order: workgroups are dispatched round-robin over the 8 XCDs (each with its own
// L2), so hardware block b runs on XCD b % 8.  Giving each XCD a contiguous range of tiles puts the
// neighbouring runs of every digit (tile t, t+1) in the same L2, where their partial lines merge
// before write-back.  Bijective for any nb.
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t nb) {
  constexpr int kXcd = 8;
  const int64_t q = nb / kXcd, r = nb % kXcd, x = b % kXcd, i = b / kXcd;
  return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// SINGLE (E <= kSortTile, one tile): the tile's own digit starts are the global ones, so the pass
// needs no count kernel and no scan — one launch per pass instead of three (the sampled blocks'
// loss transposes of ~1k pairs inside the cfg5 replay).
template <int BITS, bool HAS_B, int RR = kSortRounds, bool GEN = false, bool SINGLE = false>
__global__ void __launch_bounds__(kSortThreads) k_digit_scatter(
    const int32_t* keys_in, const int32_t* a_in, const int32_t* b_in, int64_t E, int shift,
    const int32_t* offs, int32_t* keys_out, int32_t* a_out, int32_t* b_out, int identity_a,
    KeyGen gen = KeyGen{nullptr, 0}, int32_t* gen_out = nullptr) {
  constexpr int R = 1 << BITS;
  constexpr int NW = kSortThreads / 64;
  constexpr int TILE = kSortThreads * RR;
  constexpr int PER_WAVE = TILE / NW;
  __shared__ int wcount[NW][R];                  // running count -> wave offset within tile
  __shared__ int gbase[R];                       // global start of this tile's digit run, then
                                                 // minus its tile-local start
  // (Measured and not kept, round 5: key and payload as one 8-B LDS word — reorder conflicts
  // 2.32 -> 2.12 per instruction, the cfg4 draw + sort 2.862 -> 2.866 ms.)
  __shared__ int skey[TILE];
  __shared__ int sa[TILE];
  __shared__ int sb[HAS_B ? TILE : 1];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t tile = xcd_tile(blockIdx.x, gridDim.x);
  for (int dd = threadIdx.x; dd < R; dd += kSortThreads) {
    for (int w = 0; w < NW; ++w) wcount[w][dd] = 0;
    gbase[dd] = SINGLE ? 0 : offs[(int64_t)dd * gridDim.x + tile];
  }
  __syncthreads();
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t tile0 = tile * TILE;
  const int64_t wave0 = tile0 + (int64_t)wid * PER_WAVE;
  int key[RR], rank[RR], va[RR], vb[RR];
  const uint64_t seed = GEN ? *gen.seed : 0;
  // every load of the tile issued before the ranking: the wave barriers and LDS traffic of the
  // ranking loop would otherwise keep the compiler from hoisting them, one HBM latency per round
#pragma unroll
  for (int r = 0; r < RR; ++r) {
    const int64_t i = wave0 + r * 64 + lane;
    const bool valid = i < E;
    if (GEN) {
      key[r] = valid ? uniform_draw(seed, i, gen.hi) : 0;
      if (valid && gen_out) gen_out[i] = key[r];   // the draws in position order (coalesced)
    } else {
      key[r] = valid ? keys_in[i] : 0;
    }
    va[r] = valid ? (identity_a ? (int)i : a_in[i]) : 0;
    vb[r] = (HAS_B && valid) ? b_in[i] : 0;
  }
#pragma unroll
  for (int r = 0; r < RR; ++r) {
    const int64_t i = wave0 + r * 64 + lane;
    const bool valid = i < E;
    const int digit = (key[r] >> shift) & (R - 1);
    unsigned long long match = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < BITS; ++bit) {
      const unsigned long long m = __ballot((digit >> bit) & 1);
      match &= ((digit >> bit) & 1) ? m : ~m;
    }
    // only the first lane of each digit group reads the wave's running count; the others get
    // it from that lane by ds_bpermute (64 random LDS reads per round become ~40; round 5:
    // 2.884 -> 2.872 ms for the cfg4 negatives)
    const int below = __popcll(match & lt_mask);
    const bool leader = valid && below == 0;
    int before = leader ? wcount[wid][digit] : 0;        // the group's first lane reads ...
    const int src = valid ? (int)__builtin_ctzll(match) : lane;
    before = __builtin_amdgcn_ds_bpermute(src << 2, before);   // ... and hands it to the group
    rank[r] = valid ? before + below : -1;
    __builtin_amdgcn_wave_barrier();
    if (leader) wcount[wid][digit] = before + __popcll(match);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // tile-local digit starts (exclusive scan over digits of the tile totals) and wave offsets
  {
    __shared__ int part[kSortThreads];
    constexpr int DPT = (R + kSortThreads - 1) / kSortThreads;   // digits per thread (1 or 2)
    int tot[DPT], s = 0;
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const int dd = threadIdx.x * DPT + q;
      int t = 0;
      if (dd < R)
        for (int w = 0; w < NW; ++w) t += wcount[w][dd];
      tot[q] = t;
      s += t;
    }
    part[threadIdx.x] = s;
    __syncthreads();
    // Hillis-Steele inclusive scan of the kSortThreads per-thread sums
    for (int o = 1; o < kSortThreads; o <<= 1) {
      const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    int run = part[threadIdx.x] - s;
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const int dd = threadIdx.x * DPT + q;
      if (dd < R) {
        // the run's global start minus its tile start: one lookup per item (SINGLE: both equal)
        if (!SINGLE) gbase[dd] -= run;
        int o = run;
        for (int w = 0; w < NW; ++w) {
          const int c = wcount[w][dd];
          wcount[w][dd] = o;
          o += c;
        }
      }
      run += tot[q];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RR; ++r) {
    if (rank[r] >= 0) {
      const int digit = (key[r] >> shift) & (R - 1);
      const int pos = wcount[wid][digit] + rank[r];
      skey[pos] = key[r];
      sa[pos] = va[r];
      if (HAS_B) sb[pos] = vb[r];
    }
  }
  __syncthreads();
  const int n_tile = (int)min<int64_t>(TILE, E - tile0);
  for (int j = threadIdx.x; j < n_tile; j += kSortThreads) {
    const int k = skey[j];
    const int digit = (k >> shift) & (R - 1);
    const int64_t pos = (int64_t)gbase[digit] + j;
    keys_out[pos] = k;
    a_out[pos] = sa[j];
    if (HAS_B) b_out[pos] = sb[j];
  }
}

// rowptr[r] = #sorted keys < r for r in [0, n_keys] (keys == n_keys are dropped sentinels).
// rowptr[r] = lower_bound(skey, r) for r in [0, n_keys]: one thread per row, a binary search over
// the sorted keys (the sentinel n_keys of dropped edges sorts last, so rowptr[n_keys] = valid
// edges).  Every thread does ~log2(E) cached reads; no thread ever fills a run of empty rows
// serially, which the per-edge boundary scheme did (a graph whose keys leave a long tail of
// empty rows made one thread write them all).
__global__ void __launch_bounds__(256) k_rowptr_from_sorted(const int32_t* skey, int64_t E,
                                                            int64_t n_keys, int32_t* rowptr) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > n_keys) return;
  int64_t lo = 0, hi = E;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (skey[mid] < r) lo = mid + 1;
    else hi = mid;
  }
  rowptr[r] = (int32_t)lo;
}

__global__ void __launch_bounds__(256) k_gather_other(const int32_t* perm, const int32_t* skey,
                                                      const int64_t* other, int64_t E,
                                                      int64_t n_keys, int32_t* col) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < E) col[i] = skey[i] < n_keys ? (int32_t)other[perm[i]] : 0;
}

// key32 = key if in [0, n_keys) else n_keys (sentinel); counts invalid keys.
__global__ void __launch_bounds__(256) k_prepare_keys32(const int32_t* key, int64_t E,
                                                        int64_t n_keys, int32_t* key32,
                                                        int32_t* invalid) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int bad = 0;
  if (i < E) {
    int32_t k = key[i];
    bool ok = k >= 0 && k < n_keys;
    key32[i] = ok ? k : (int32_t)n_keys;
    bad = ok ? 0 : 1;
  }
  unsigned long long m = __ballot(bad);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(invalid, __popcll(m));
}

// int64 keys -> int32 key32 (out-of-range -> n_keys sentinel); counts invalid keys.
__global__ void __launch_bounds__(256) k_prepare_keys64(const int64_t* key, int64_t E,
                                                        int64_t n_keys, int32_t* key32,
                                                        int32_t* invalid) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int bad = 0;
  if (i < E) {
    const int64_t k = key[i];
    const bool ok = k >= 0 && k < n_keys;
    key32[i] = ok ? (int32_t)k : (int32_t)n_keys;
    bad = ok ? 0 : 1;
  }
  unsigned long long m = __ballot(bad);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(invalid, __popcll(m));
}

__global__ void k_fill_i32(int32_t* p, int64_t n, int32_t v) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// Digit width: the one of 6..9 bits minimising passes x measured per-pass time (counts + scan +
// scatter, 20M pairs on MI355X: 6 bits 108 us, 7 bits 117, 8 bits 147, 9 bits 183 — measured in
// round 1 on the then 4096-item tile; fewer digits mean longer per-digit runs per tile, so a
// 6-bit pass writes ~256-B runs where a 9-bit one writes ~32-B runs, twice that on today's
// kSortTile of 8192).  The planner still chooses 7 + 7 + 6 bits for the cfg4 negatives, which the
// round-4 A/B on the 8192-item tile confirmed (scripts/gpu_sort_ab.sh).  17-bit post ids: 3 passes of 6 (339 us) beat 2 of 9 (381); 20-bit:
// 3 of 7.  (10-bit digits, 2 passes for 19-20-bit ids, were measured slower than 3 passes of 8.)
// Small sorts (fewer than kSmallSort pairs: a sampled block's transposes, ~0.1M edges) are
// bound by their launches (count, scan, scatter per pass), not by the ranking: the fewest passes
// of up to 10 bits (cfg5: 17-bit local ids in 2 passes instead of 3).
constexpr int64_t kSmallSort = int64_t(1) << 20;
static void radix_plan(int64_t n_keys, int64_t E, int* passes, int* bits) {
  int b = 0;
  while ((int64_t(1) << b) <= n_keys) ++b;   // keys in [0, n_keys] incl. sentinel
  static const int cost[10] = {0, 0, 0, 0, 0, 0, 108, 117, 147, 183};
  int best = 6, best_cost = 1 << 30;
  for (int d = 6; d <= 9; ++d) {
    const int c = ((b + d - 1) / d) * cost[d];
    if (c < best_cost) best_cost = c, best = d;
  }
  if (E < kSmallSort) {
    const int np = std::max(1, (b + 9) / 10);
    best = std::max(6, std::min(10, (b + np - 1) / np));
  }
  *bits = best;
  *passes = (b + best - 1) / best;
  static const int forced = getenv("HGNN_SORT_BITS") ? atoi(getenv("HGNN_SORT_BITS")) : 0;
  if (forced >= 6 && forced <= 10) {   // measurement override
    *bits = forced;
    *passes = (b + forced - 1) / forced;
  }
  if (*passes < 1) *passes = 1;
}

#define HGNN_BITS_SWITCH(bits, M) \
  switch (bits) {                 \
    case 6: M(6); break;          \
    case 7: M(7); break;          \
    case 8: M(8); break;          \
    case 10: M(10); break;        \
    default: M(9); break;         \
  }

static size_t sort_ws_bytes(int64_t E) {
  int64_t nb = cdiv(E, kSortTile);
  size_t scan_b = 0;
  exclusive_scan_i32(nullptr, nullptr, nb * kMaxRadix, nullptr, &scan_b, 0);
  return 5 * align_up((size_t)E * 4, 256) + 2 * align_up((size_t)(nb * kMaxRadix + 1) * 4, 256) +
         scan_b + 2048;
}

// LSD sort of prepared keys (ka, values in [0, n_keys]) with payload a (identity if a_in null)
// and optional b.  The last pass lands the payloads in a_out / b_out; the sorted keys end in
// *k_sorted (a workspace buffer).
static int radix_sort_pairs(const int32_t* k_in, int32_t* ka, int64_t E, int64_t n_keys,
                            const int32_t* a_in, const int32_t* b_in, int32_t* a_out,
                            int32_t* b_out, Workspace& w, hipStream_t stream,
                            const int32_t** k_sorted, KeyGen gen = KeyGen{nullptr, 0},
                            int32_t* gen_out = nullptr) {
  int32_t* kb = w.take<int32_t>(E);
  int32_t* ta = w.take<int32_t>(E);
  int32_t* tb = b_in ? w.take<int32_t>(E) : nullptr;
  const int64_t nb = cdiv(E, kSortTile);
  int32_t* counts = w.take<int32_t>(nb * kMaxRadix + 1);
  int32_t* offs = w.take<int32_t>(nb * kMaxRadix + 1);
  int passes, bits;
  radix_plan(n_keys, E, &passes, &bits);
  // the last pass takes only the bits left (>= 6: narrower digits measured no faster), e.g. 7 + 7
  // + 6 for 20-bit keys: fewer ranking ballots and longer runs per digit in its scatter
  int key_bits = 0;
  while ((int64_t(1) << key_bits) <= n_keys) ++key_bits;
  const int last_bits = std::max(6, std::min(bits, key_bits - bits * (passes - 1)));
  const int64_t ncount = nb * ((int64_t)1 << bits);
  size_t scan_b = 0;
  exclusive_scan_i32(nullptr, nullptr, ncount, nullptr, &scan_b, stream);
  void* scan_ws = w.take<char>(scan_b);
  if (!scan_ws) return fail(HGNN_E_WS, "radix sort: workspace too small");
  const int32_t* kin = k_in;   // read-only input; passes ping-pong between ka and kb
  const int32_t* ain = a_in;
  const int32_t* bin = b_in;
  for (int p = 0; p < passes; ++p) {
    const int shift = bits * p;
    const int pbits = p == passes - 1 ? last_bits : bits;
    const int64_t pcount = nb * ((int64_t)1 << pbits);
    const bool to_out = ((passes - 1 - p) % 2) == 0;
    int32_t* kout = (kin == ka) ? kb : ka;   // (k_in itself is never written)
    int32_t* aout = to_out ? a_out : ta;
    int32_t* bout = b_in ? (to_out ? b_out : tb) : nullptr;
    const int ident = (p == 0 && a_in == nullptr) ? 1 : 0;
    const bool g0 = p == 0 && gen.seed != nullptr;   // first pass: keys drawn, not loaded
    const bool single = nb == 1;                     // one tile: no counts, no scan
#define HGNN_COUNTS(BV)                                                                           \
  if (g0) hipLaunchKernelGGL((k_digit_counts<BV, kSortRounds, true>), dim3(nb), dim3(kSortThreads), \
                             0, stream, kin, E, shift, counts, gen);                              \
  else hipLaunchKernelGGL((k_digit_counts<BV>), dim3(nb), dim3(kSortThreads), 0, stream, kin, E,  \
                          shift, counts, KeyGen{nullptr, 0})
    if (!single) {
      HGNN_BITS_SWITCH(pbits, HGNN_COUNTS)
      if (int rc = check_launch("k_digit_counts")) return rc;
      if (int rc = exclusive_scan_i32(counts, offs, pcount, scan_ws, &scan_b, stream)) return rc;
    }
#undef HGNN_COUNTS
#define HGNN_SCATTER(BV, HB, SG)                                                              \
  hipLaunchKernelGGL((k_digit_scatter<BV, HB, kSortRounds, false, SG>), dim3(nb),               \
                     dim3(kSortThreads), 0, stream, kin, ain, bin, E, shift, offs, kout, aout,   \
                     bout, ident)
#define HGNN_SCATTER_G(BV, SG)                                                                \
  hipLaunchKernelGGL((k_digit_scatter<BV, false, kSortRounds, true, SG>), dim3(nb),             \
                     dim3(kSortThreads), 0, stream, kin, ain, bin, E, shift, offs, kout, aout,   \
                     bout, ident, gen, gen_out)
#define HGNN_SCATTER_B(BV)                                                                    \
  if (g0) {                                                                                   \
    if (single) { HGNN_SCATTER_G(BV, true); } else { HGNN_SCATTER_G(BV, false); }             \
  } else if (b_in) {                                                                          \
    if (single) { HGNN_SCATTER(BV, true, true); } else { HGNN_SCATTER(BV, true, false); }     \
  } else {                                                                                    \
    if (single) { HGNN_SCATTER(BV, false, true); } else { HGNN_SCATTER(BV, false, false); }   \
  }
    HGNN_BITS_SWITCH(pbits, HGNN_SCATTER_B)
#undef HGNN_SCATTER_B
#undef HGNN_SCATTER_G
#undef HGNN_SCATTER
    if (int rc = check_launch("k_digit_scatter")) return rc;
    kin = kout;
    ain = aout;
    bin = bout;
  }
  *k_sorted = kin;
  return HGNN_OK;
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_version(void) { return 101; }

const char* hgnn_last_error_string(void) { return g_err; }

size_t hgnn_coo_to_csr_ws_bytes(int64_t E, int64_t n_keys) {
  (void)n_keys;
  return sort_ws_bytes(E < 1 ? 1 : E);
}

int hgnn_coo_to_csr(const int64_t* key, const int64_t* other, int64_t E, int64_t n_keys,
                    int64_t n_other, int32_t* rowptr, int32_t* col, int32_t* perm,
                    int32_t* d_invalid, void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (E < 0 || E >= (int64_t(1) << 31) - 1 || n_keys < 0 || n_keys >= (int64_t(1) << 31) - 1)
    return fail(HGNN_E_ARG, "coo_to_csr: E=%lld n_keys=%lld out of range", (long long)E,
                (long long)n_keys);
  if (!rowptr || !d_invalid || (E > 0 && (!key || !other || !col || !perm)))
    return fail(HGNN_E_ARG, "coo_to_csr: null pointer");
  (void)hipMemsetAsync(d_invalid, 0, sizeof(int32_t), stream);
  if (E == 0 || n_keys == 0) {
    hipLaunchKernelGGL(k_fill_i32, dim3(cdiv(n_keys + 1, 256)), dim3(256), 0, stream, rowptr,
                       n_keys + 1, 0);
    if (E > 0)  // every edge is out of range
      hipLaunchKernelGGL(k_prepare_keys, dim3(cdiv(E, 256)), dim3(256), 0, stream, key, other,
                         E, n_keys, n_other, col, d_invalid);
    return check_launch("coo_to_csr(empty)");
  }
  if (ws_bytes < sort_ws_bytes(E)) return fail(HGNN_E_WS, "coo_to_csr: workspace too small");
  Workspace w(ws, ws_bytes);
  int32_t* ka = w.take<int32_t>(E);
  hipLaunchKernelGGL(k_prepare_keys, dim3(cdiv(E, 256)), dim3(256), 0, stream, key, other, E,
                     n_keys, n_other, ka, d_invalid);
  if (int rc = check_launch("k_prepare_keys")) return rc;
  const int32_t* sk = nullptr;
  if (int rc = radix_sort_pairs(ka, ka, E, n_keys, nullptr, nullptr, perm, nullptr, w, stream,
                                &sk))
    return rc;
  hipLaunchKernelGGL(k_rowptr_from_sorted, dim3(cdiv(n_keys + 1, 256)), dim3(256), 0, stream, sk, E,
                     n_keys, rowptr);
  if (int rc = check_launch("k_rowptr_from_sorted")) return rc;
  hipLaunchKernelGGL(k_gather_other, dim3(cdiv(E, 256)), dim3(256), 0, stream, perm, sk, other,
                     E, n_keys, col);
  return check_launch("k_gather_other");
}

size_t hgnn_sort_pairs_ws_bytes(int64_t E, int64_t n_keys) {
  (void)n_keys;
  return sort_ws_bytes(E < 1 ? 1 : E);
}

int hgnn_sort_pairs_i32(const int32_t* keys, const int32_t* a, const int32_t* b, int64_t E,
                        int64_t n_keys, int32_t* rowptr, int32_t* a_sorted, int32_t* b_sorted,
                        int32_t* d_invalid, void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (E < 0 || E >= (int64_t(1) << 31) - 1 || n_keys < 0 || n_keys >= (int64_t(1) << 31) - 1)
    return fail(HGNN_E_ARG, "sort_pairs: E=%lld n_keys=%lld out of range", (long long)E,
                (long long)n_keys);
  if (!rowptr || (E > 0 && (!keys || !a || !a_sorted || (b && !b_sorted))))
    return fail(HGNN_E_ARG, "sort_pairs: null pointer");
  if (d_invalid) (void)hipMemsetAsync(d_invalid, 0, sizeof(int32_t), stream);
  if (E == 0 || n_keys == 0) {
    hipLaunchKernelGGL(k_fill_i32, dim3(cdiv(n_keys + 1, 256)), dim3(256), 0, stream, rowptr,
                       n_keys + 1, 0);
    return check_launch("sort_pairs(empty)");
  }
  if (ws_bytes < sort_ws_bytes(E)) return fail(HGNN_E_WS, "sort_pairs: workspace too small");
  Workspace w(ws, ws_bytes);
  int32_t* ka = w.take<int32_t>(E);
  const int32_t* kin = keys;   // d_invalid == NULL: the caller guarantees keys in [0, n_keys)
  if (d_invalid) {
    hipLaunchKernelGGL(k_prepare_keys32, dim3(cdiv(E, 256)), dim3(256), 0, stream, keys, E,
                       n_keys, ka, d_invalid);
    if (int rc = check_launch("k_prepare_keys32")) return rc;
    kin = ka;
  }
  const int32_t* sk = nullptr;
  if (int rc = radix_sort_pairs(kin, ka, E, n_keys, a, b, a_sorted, b_sorted, w, stream, &sk))
    return rc;
  hipLaunchKernelGGL(k_rowptr_from_sorted, dim3(cdiv(n_keys + 1, 256)), dim3(256), 0, stream, sk, E,
                     n_keys, rowptr);
  return check_launch("k_rowptr_from_sorted");
}

}  // extern "C"

namespace hgnn {
// CSC entry i of a CSR: its row (binary search of the CSR position t_perm[i] in rowptr) and, if
// asked, 1/deg of that row — the weight K2 streams (graph.RelationCSR.bwd_weights).
__global__ void k_transpose_finish(const int32_t* rowptr, int64_t n_rows, const int32_t* t_perm,
                                   int64_t E, int32_t* t_col, float* t_w) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E) return;
  const int32_t pos = t_perm[i];
  int64_t lo = 0, hi = n_rows;   // rowptr[lo] <= pos < rowptr[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (rowptr[mid] <= pos) lo = mid; else hi = mid;
  }
  t_col[i] = (int32_t)lo;
  if (t_w) t_w[i] = 1.f / (float)(rowptr[lo + 1] - rowptr[lo]);
}
}  // namespace hgnn

extern "C" {

int hgnn_csr_transpose(const int32_t* rowptr, const int32_t* col, int64_t n_rows, int64_t E,
                       int64_t n_cols, int32_t* t_rowptr, int32_t* t_col, int32_t* t_perm,
                       float* t_w, void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (E < 0 || E >= (int64_t(1) << 31) - 1 || n_rows < 0 || n_cols < 0 ||
      n_cols >= (int64_t(1) << 31) - 1)
    return fail(HGNN_E_ARG, "csr_transpose: E=%lld n_rows=%lld n_cols=%lld out of range",
                (long long)E, (long long)n_rows, (long long)n_cols);
  if (!t_rowptr || (E > 0 && (!rowptr || !col || !t_col || !t_perm)))
    return fail(HGNN_E_ARG, "csr_transpose: null pointer");
  if (E == 0 || n_cols == 0) {
    hipLaunchKernelGGL(k_fill_i32, dim3(cdiv(n_cols + 1, 256)), dim3(256), 0, stream, t_rowptr,
                       n_cols + 1, 0);
    return check_launch("csr_transpose(empty)");
  }
  if (ws_bytes < sort_ws_bytes(E)) return fail(HGNN_E_WS, "csr_transpose: workspace too small");
  Workspace w(ws, ws_bytes);
  int32_t* ka = w.take<int32_t>(E);
  const int32_t* sk = nullptr;
  // payload: the CSR position itself (identity on the first pass), no key validation pass
  if (int rc = radix_sort_pairs(col, ka, E, n_cols, nullptr, nullptr, t_perm, nullptr, w, stream,
                                &sk))
    return rc;
  hipLaunchKernelGGL(k_rowptr_from_sorted, dim3(cdiv(n_cols + 1, 256)), dim3(256), 0, stream, sk,
                     E, n_cols, t_rowptr);
  if (int rc = check_launch("k_rowptr_from_sorted")) return rc;
  hipLaunchKernelGGL(k_transpose_finish, dim3(cdiv(E, 256)), dim3(256), 0, stream, rowptr, n_rows,
                     t_perm, E, t_col, t_w);
  return check_launch("k_transpose_finish");
}

}  // extern "C"

namespace hgnn {
// the row owning each CSR position (binary search in rowptr)
__global__ void k_row_of_position(const int32_t* rowptr, int64_t n_rows, int64_t E,
                                  int32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E) return;
  int64_t lo = 0, hi = n_rows;   // rowptr[lo] <= i < rowptr[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (rowptr[mid] <= i) lo = mid; else hi = mid;
  }
  out[i] = (int32_t)lo;
}
}  // namespace hgnn

extern "C" {

size_t hgnn_link_group_ws_bytes(int64_t E) { return sort_ws_bytes(E < 1 ? 1 : E); }

int hgnn_link_group(const int32_t* pu, const int32_t* pp, const int32_t* pn, int64_t E,
                    int64_t n_users, int64_t n_posts, int32_t* rowptr_u, int32_t* col_p,
                    int32_t* neg, int32_t* uop, int32_t* p_rowptr, int32_t* p_users,
                    int32_t* p_perm, int32_t* n_rowptr, int32_t* n_users_sorted, void* ws,
                    size_t ws_bytes, hgnn_stream_t stream_) {
  if (E < 0 || n_users < 1 || n_posts < 1 || !uop || (E > 0 && (!pu || !pp || !pn)))
    return fail(HGNN_E_ARG, "link_group: E=%lld n_users=%lld n_posts=%lld", (long long)E,
                (long long)n_users, (long long)n_posts);
  // the pairs by user (stable: positive order within a user), their posts and negatives along
  if (int rc = hgnn_sort_pairs_i32(pu, pp, pn, E, n_users, rowptr_u, col_p, neg, nullptr, ws,
                                   ws_bytes, stream_))
    return rc;
  if (E > 0) {
    hipLaunchKernelGGL(k_row_of_position, dim3(cdiv(E, 256)), dim3(256), 0, as_stream(stream_),
                       rowptr_u, n_users, E, uop);
    if (int rc = check_launch("k_row_of_position")) return rc;
  }
  // the same pairs by post (the dU scoring pass's transpose), and the negatives by post
  if (int rc = hgnn_csr_transpose(rowptr_u, col_p, n_users, E, n_posts, p_rowptr, p_users, p_perm,
                                  nullptr, ws, ws_bytes, stream_))
    return rc;
  return hgnn_sort_pairs_i32(neg, uop, nullptr, E, n_posts, n_rowptr, n_users_sorted, nullptr,
                             nullptr, ws, ws_bytes, stream_);
}

}  // extern "C"

namespace hgnn {
// The CSCs of several destination-grouped CSRs in one sort: relation r's columns are keyed
// col + cbase[r] and its positions numbered from ebase[r], so one stable sort over the combined
// key range groups every relation's entries by (relation, column); each output then takes its
// slice, zero-based.
constexpr int kTransposeMax = 8;
struct TransposeTab {
  const int32_t* rowptr[kTransposeMax];
  const int32_t* col[kTransposeMax];
  int32_t* t_rowptr[kTransposeMax];
  int32_t* t_col[kTransposeMax];
  int32_t* t_perm[kTransposeMax];
  float* t_w[kTransposeMax];
  int64_t n_rows[kTransposeMax];
  int64_t ebase[kTransposeMax + 1];   // position offsets
  int64_t cbase[kTransposeMax + 1];   // key (column) offsets
  int32_t n;
};

__device__ __forceinline__ int tt_find(const int64_t* off, int n, int64_t i) {
  int r = 0;
  while (r + 1 < n && i >= off[r + 1]) ++r;
  return r;
}

__global__ void k_transpose_keys(const TransposeTab t, int32_t* keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.ebase[t.n]) return;
  const int r = tt_find(t.ebase, t.n, i);
  keys[i] = t.col[r][i - t.ebase[r]] + (int32_t)t.cbase[r];
}

// sorted entry i (global position p = perm_all[i]): relation r, its row (binary search in r's
// rowptr), 1/deg of the row; written at i - (first sorted index of r)
__global__ void k_transpose_finish_multi(const TransposeTab t, const int32_t* perm_all,
                                         const int32_t* rowptr_all) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.ebase[t.n]) return;
  const int64_t p = perm_all[i];
  const int r = tt_find(t.ebase, t.n, p);
  const int64_t pos = p - t.ebase[r];
  const int32_t* rp = t.rowptr[r];
  int64_t lo = 0, hi = t.n_rows[r];
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (rp[mid] <= pos) lo = mid; else hi = mid;
  }
  const int64_t j = i - rowptr_all[t.cbase[r]];
  t.t_col[r][j] = (int32_t)lo;
  t.t_perm[r][j] = (int32_t)pos;
  if (t.t_w[r]) t.t_w[r][j] = 1.f / (float)(rp[lo + 1] - rp[lo]);
}

__global__ void k_transpose_rowptr_split(const TransposeTab t, const int32_t* rowptr_all) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // entry j of relation r
  if (g >= t.cbase[t.n] + t.n) return;                                // sits at cbase[r] + r + j
  int r = 0;
  while (r + 1 < t.n && g >= t.cbase[r + 1] + r + 1) ++r;
  const int64_t j = g - t.cbase[r] - r;
  t.t_rowptr[r][j] = rowptr_all[t.cbase[r] + j] - rowptr_all[t.cbase[r]];
}
}  // namespace hgnn

extern "C" {

size_t hgnn_csr_transpose_multi_ws_bytes(int64_t E_total, int64_t n_cols_total) {
  const int64_t E = E_total < 1 ? 1 : E_total;
  return sort_ws_bytes(E) + 2 * align_up((size_t)E * 4, 256) +
         align_up((size_t)(n_cols_total + 1) * 4, 256) + 512;
}

int hgnn_csr_transpose_multi(int32_t n_rel, const int32_t* const* rowptr,
                             const int32_t* const* col, const int64_t* n_rows, const int64_t* E,
                             const int64_t* n_cols, int32_t* const* t_rowptr,
                             int32_t* const* t_col, int32_t* const* t_perm, float* const* t_w,
                             void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_rel < 1 || n_rel > kTransposeMax || !rowptr || !col || !n_rows || !E || !n_cols ||
      !t_rowptr || !t_col || !t_perm)
    return fail(HGNN_E_ARG, "csr_transpose_multi: n_rel=%d (1..%d) or null array", n_rel,
                kTransposeMax);
  TransposeTab t{};
  t.n = n_rel;
  for (int r = 0; r < n_rel; ++r) {
    if (E[r] < 0 || n_rows[r] < 0 || n_cols[r] < 0 || !t_rowptr[r] ||
        (E[r] > 0 && (!rowptr[r] || !col[r] || !t_col[r] || !t_perm[r])))
      return fail(HGNN_E_ARG, "csr_transpose_multi: relation %d", r);
    t.rowptr[r] = rowptr[r]; t.col[r] = col[r]; t.n_rows[r] = n_rows[r];
    t.t_rowptr[r] = t_rowptr[r]; t.t_col[r] = t_col[r]; t.t_perm[r] = t_perm[r];
    t.t_w[r] = t_w ? t_w[r] : nullptr;
    t.ebase[r + 1] = t.ebase[r] + E[r];
    t.cbase[r + 1] = t.cbase[r] + n_cols[r];
  }
  const int64_t Et = t.ebase[n_rel], K = t.cbase[n_rel];
  if (Et >= (int64_t(1) << 31) - 1 || K >= (int64_t(1) << 31) - 1)
    return fail(HGNN_E_ARG, "csr_transpose_multi: E=%lld keys=%lld out of range",
                (long long)Et, (long long)K);
  if (ws_bytes < hgnn_csr_transpose_multi_ws_bytes(Et, K))
    return fail(HGNN_E_WS, "csr_transpose_multi: workspace too small");
  Workspace w(ws, ws_bytes);
  int32_t* keys = w.take<int32_t>(Et < 1 ? 1 : Et);
  int32_t* perm = w.take<int32_t>(Et < 1 ? 1 : Et);
  int32_t* rp_all = w.take<int32_t>(K + 1);
  if (Et > 0 && K > 0) {
    hipLaunchKernelGGL(k_transpose_keys, dim3(cdiv(Et, 256)), dim3(256), 0, stream, t, keys);
    if (int rc = check_launch("k_transpose_keys")) return rc;
    int32_t* ka = w.take<int32_t>(Et);
    const int32_t* sk = nullptr;
    if (int rc = radix_sort_pairs(keys, ka, Et, K, nullptr, nullptr, perm, nullptr, w, stream,
                                  &sk))
      return rc;
    hipLaunchKernelGGL(k_rowptr_from_sorted, dim3(cdiv(K + 1, 256)), dim3(256), 0, stream, sk,
                       Et, K, rp_all);
    if (int rc = check_launch("k_rowptr_from_sorted")) return rc;
    hipLaunchKernelGGL(k_transpose_finish_multi, dim3(cdiv(Et, 256)), dim3(256), 0, stream, t,
                       perm, rp_all);
    if (int rc = check_launch("k_transpose_finish_multi")) return rc;
  } else {
    hipLaunchKernelGGL(k_fill_i32, dim3(cdiv(K + 1, 256)), dim3(256), 0, stream, rp_all, K + 1,
                       0);
  }
  hipLaunchKernelGGL(k_transpose_rowptr_split, dim3(cdiv(K + n_rel, 256)), dim3(256), 0, stream,
                     t, rp_all);
  return check_launch("k_transpose_rowptr_split");
}

int hgnn_draw_sort_negatives(const uint64_t* d_seed, const int32_t* a, int64_t E, int64_t n_keys,
                             int32_t* neg_out, int32_t* rowptr, int32_t* a_sorted, void* ws,
                             size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (E < 0 || E >= (int64_t(1) << 31) - 1 || n_keys < 1 || n_keys >= (int64_t(1) << 31) - 1)
    return fail(HGNN_E_ARG, "draw_sort_negatives: E=%lld n_keys=%lld out of range", (long long)E,
                (long long)n_keys);
  if (!rowptr || (E > 0 && (!d_seed || !a || !a_sorted)))
    return fail(HGNN_E_ARG, "draw_sort_negatives: null pointer");
  if (E == 0) {
    hipLaunchKernelGGL(k_fill_i32, dim3(cdiv(n_keys + 1, 256)), dim3(256), 0, stream, rowptr,
                       n_keys + 1, 0);
    return check_launch("draw_sort_negatives(empty)");
  }
  if (ws_bytes < sort_ws_bytes(E))
    return fail(HGNN_E_WS, "draw_sort_negatives: workspace too small");
  Workspace w(ws, ws_bytes);
  int32_t* ka = w.take<int32_t>(E);
  const int32_t* sk = nullptr;
  // the draws are < n_keys by construction: no sentinel value to leave room for
  if (int rc = radix_sort_pairs(nullptr, ka, E, n_keys - 1, a, nullptr, a_sorted, nullptr, w, stream,
                                &sk, KeyGen{d_seed, (uint32_t)n_keys}, neg_out))
    return rc;
  hipLaunchKernelGGL(k_rowptr_from_sorted, dim3(cdiv(n_keys + 1, 256)), dim3(256), 0, stream, sk, E,
                     n_keys, rowptr);
  return check_launch("k_rowptr_from_sorted");
}

int hgnn_sort_pairs_i64(const int64_t* keys, const int32_t* a, const int32_t* b, int64_t E,
                        int64_t n_keys, int32_t* rowptr, int32_t* a_sorted, int32_t* b_sorted,
                        int32_t* d_invalid, void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (E < 0 || E >= (int64_t(1) << 31) - 1 || n_keys < 0 || n_keys >= (int64_t(1) << 31) - 1)
    return fail(HGNN_E_ARG, "sort_pairs_i64: E=%lld n_keys=%lld out of range", (long long)E,
                (long long)n_keys);
  if (!rowptr || !d_invalid || (E > 0 && (!keys || !a || !a_sorted || (b && !b_sorted))))
    return fail(HGNN_E_ARG, "sort_pairs_i64: null pointer");
  (void)hipMemsetAsync(d_invalid, 0, sizeof(int32_t), stream);
  if (E == 0 || n_keys == 0) {
    hipLaunchKernelGGL(k_fill_i32, dim3(cdiv(n_keys + 1, 256)), dim3(256), 0, stream, rowptr,
                       n_keys + 1, 0);
    if (E > 0)
      hipLaunchKernelGGL(k_prepare_keys64, dim3(cdiv(E, 256)), dim3(256), 0, stream, keys, E,
                         n_keys, a_sorted, d_invalid);   // (count only; payloads are undefined)
    return check_launch("sort_pairs_i64(empty)");
  }
  if (ws_bytes < sort_ws_bytes(E)) return fail(HGNN_E_WS, "sort_pairs_i64: workspace too small");
  Workspace w(ws, ws_bytes);
  int32_t* ka = w.take<int32_t>(E);
  hipLaunchKernelGGL(k_prepare_keys64, dim3(cdiv(E, 256)), dim3(256), 0, stream, keys, E, n_keys,
                     ka, d_invalid);
  if (int rc = check_launch("k_prepare_keys64")) return rc;
  const int32_t* sk = nullptr;
  if (int rc = radix_sort_pairs(ka, ka, E, n_keys, a, b, a_sorted, b_sorted, w, stream, &sk))
    return rc;
  hipLaunchKernelGGL(k_rowptr_from_sorted, dim3(cdiv(n_keys + 1, 256)), dim3(256), 0, stream, sk, E,
                     n_keys, rowptr);
  return check_launch("k_rowptr_from_sorted");
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// Degree-skew plan and 1/deg.
// ------------------------------------------------------------------------------------------
namespace hgnn {

__global__ void k_plan_flags(const int32_t* rowptr, int64_t n, int32_t chunk, int32_t* heavy,
                             int32_t* nch) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t deg = rowptr[i + 1] - rowptr[i];
  bool h = deg > chunk;
  heavy[i] = h ? 1 : 0;
  nch[i] = h ? (deg + chunk - 1) / chunk : 0;
}

__global__ void k_plan_counts(const int32_t* hscan, const int32_t* cscan, int64_t n,
                              int32_t* out2) {
  out2[0] = hscan[n];
  out2[1] = cscan[n];
}

__global__ void k_plan_scatter(const int32_t* heavy, const int32_t* hscan, const int32_t* cscan,
                               int64_t n, int32_t* heavy_rows, int32_t* heavy_first) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && heavy[i]) {
    heavy_rows[hscan[i]] = (int32_t)i;
    heavy_first[hscan[i]] = cscan[i];
  }
  if (i == n) heavy_first[hscan[n]] = cscan[n];
}

__global__ void k_inv_degree(const int32_t* rowptr, int64_t n, float* inv) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t deg = rowptr[i + 1] - rowptr[i];
  inv[i] = deg > 0 ? 1.0f / (float)deg : 0.0f;
}

static int plan_common(const int32_t* rowptr, int64_t n, int32_t chunk, void* ws, size_t ws_bytes,
                       hipStream_t stream, int32_t** heavy, int32_t** hscan, int32_t** cscan) {
  if (!rowptr || n < 0 || chunk <= 0) return fail(HGNN_E_ARG, "plan: bad arguments");
  Workspace w(ws, ws_bytes);
  *heavy = w.take<int32_t>(n + 1);
  int32_t* nch = w.take<int32_t>(n + 1);
  *hscan = w.take<int32_t>(n + 1);
  *cscan = w.take<int32_t>(n + 1);
  size_t sb = 0;
  exclusive_scan_i32(nullptr, nullptr, n, nullptr, &sb, stream);
  void* sws = w.take<char>(sb);
  if (!sws) return fail(HGNN_E_WS, "plan: workspace too small");
  if (n > 0) {
    hipLaunchKernelGGL(k_plan_flags, dim3(cdiv(n, 256)), dim3(256), 0, stream, rowptr, n, chunk,
                       *heavy, nch);
    if (int rc = check_launch("k_plan_flags")) return rc;
  }
  if (int rc = exclusive_scan_i32(*heavy, *hscan, n, sws, &sb, stream)) return rc;
  return exclusive_scan_i32(nch, *cscan, n, sws, &sb, stream);
}

}  // namespace hgnn

extern "C" {

size_t hgnn_plan_ws_bytes(int64_t n_rows) {
  size_t sb = 0;
  exclusive_scan_i32(nullptr, nullptr, n_rows, nullptr, &sb, 0);
  return 4 * align_up((size_t)(n_rows + 1) * 4, 256) + sb + 2048;
}

int hgnn_plan_count(const int32_t* rowptr, int64_t n_rows, int32_t chunk, int32_t* d_counts2,
                    void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  int32_t *heavy, *hscan, *cscan;
  if (int rc = plan_common(rowptr, n_rows, chunk, ws, ws_bytes, stream, &heavy, &hscan, &cscan))
    return rc;
  hipLaunchKernelGGL(k_plan_counts, dim3(1), dim3(1), 0, stream, hscan, cscan, n_rows, d_counts2);
  return check_launch("k_plan_counts");
}

int hgnn_plan_fill(const int32_t* rowptr, int64_t n_rows, int32_t chunk, int32_t* heavy_rows,
                   int32_t* heavy_first, void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  int32_t *heavy, *hscan, *cscan;
  if (int rc = plan_common(rowptr, n_rows, chunk, ws, ws_bytes, stream, &heavy, &hscan, &cscan))
    return rc;
  hipLaunchKernelGGL(k_plan_scatter, dim3(cdiv(n_rows + 1, 256)), dim3(256), 0, stream, heavy,
                     hscan, cscan, n_rows, heavy_rows, heavy_first);
  return check_launch("k_plan_scatter");
}

int hgnn_inv_degree(const int32_t* rowptr, int64_t n_rows, float* inv_deg,
                    hgnn_stream_t stream_) {
  if (n_rows <= 0) return HGNN_OK;
  if (!rowptr || !inv_deg) return fail(HGNN_E_ARG, "inv_degree: null pointer");
  hipLaunchKernelGGL(k_inv_degree, dim3(cdiv(n_rows, 256)), dim3(256), 0, as_stream(stream_),
                     rowptr, n_rows, inv_deg);
  return check_launch("k_inv_degree");
}

}  // extern "C"
