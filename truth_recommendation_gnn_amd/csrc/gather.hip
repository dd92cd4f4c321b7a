// K1 / K2: segmented gather-reduce over a CSR — the E x d heart of SAGE mean aggregation.
//
//   out[i,:] (+)= s_i * sum_{p in row i} w_p * x[col[p], :]
//
// HBM-bound (algorithmic bytes per edge: 4 B index + 4*d B source row [+ 4 B weight]).
// Mapping (wave64, one item per wave):
//   * a row of d floats is read by LPR lanes, 16 B (float4) per lane and VPL vectors per lane,
//     so a wave covers NS = 64/LPR rows per load instruction (d=64: 4 rows x 256 B = 1 KiB);
//   * the wave pulls 64 column indices (and weights) of its row with one coalesced load, then
//     each slot of LPR lanes takes every NS-th edge, UNROLL rows in flight per slot;
//   * slots are combined with xor-shuffles; the first slot writes the row (full 256-B lines).
// No atomics: each destination row is owned by one wave, so sums are deterministic.  Rows longer
// than `chunk` edges (power-law heads) are split by the plan into chunk-sized items whose
// partial sums go to a slab, then k_fixup adds them in chunk order.
#include "hgnn_common.h"

// Cache policy of the gathered rows and the output rows (set per launch from the table sizes,
// `nt_policy` below): nt loads / stores when the table is far larger than the caches.
#include <stdlib.h>

namespace hgnn {

struct GatherArgs {
  const float* x;
  const int32_t* rowptr;
  const int32_t* col;
  const float* edge_w;
  const float* col_w;
  const float* row_w;          // per-row output scale (replaces the mean's 1/segment length)
  const int32_t* heavy_rows;
  const int32_t* heavy_first;
  float* slab;
  float* out;
  int64_t n_rows;
  int64_t n_heavy;
  int64_t n_items;
  int32_t d;
  int32_t chunk;
  int32_t mean;
  int32_t accumulate;
  int64_t acc_limit;           // > 0: only rows below it accumulate, the others are written
                               // fresh (a K2 whose output holds a root-gradient prefix)
  // score mode (hgnn_score_gather): w_p = f(<x[col[p]], rowvec[row]>) recomputed per edge
  const float* rowvec;
  const float* cscale;
  float inv_e;
  int32_t score;               // 1: c*inv_e*(sigmoid(s)-1)   2: inv_e*sigmoid(s)
  // hgnn_score_gather2: a second grouped list (the negatives, mode 2, no heavy-row plan) summed
  // into the same rows in the same pass; null otherwise
  const int32_t* rowptr2;
  int32_t nt_load;             // rows gathered with nt loads (score gathers over multi-GB tables)
  int32_t nt_store;            // output rows stored with nt stores
  const int32_t* col2;
};

// Sum of row segment [beg, end) of `col` into acc (per lane: VPL vectors of width W; each slot of
// LPR lanes holds its own partial sum, combined by slot_combine).  SC: the weight of each edge is
// recomputed from the score <x[col[p]], rv> (rv = the row's own vector, e.g. P[post] for the loss
// gradient dP) with weight mode `score`, so no per-edge weight array is stored or read.
template <int LPR, int VPL, int W, int UNROLL, bool HAS_W, bool SC>
__device__ __forceinline__ void segment_sum(const GatherArgs& a, const int32_t* col, int score,
                                            int64_t beg, int64_t end,
                                            const typename Vec<W>::T (&rv)[VPL],
                                            typename Vec<W>::T (&acc)[VPL]) {
  using V = Vec<W>;
  constexpr int NS = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int slot = lane / LPR, sl = lane % LPR;
  const int d = a.d;
  for (int64_t base = beg; base < end; base += 64) {
    const int n = (int)min<int64_t>(64, end - base);
    int cidx = 0;
    float wv = 1.f;
    if (lane < n) {
      cidx = col[base + lane];
      if (HAS_W) {
        wv = a.edge_w ? a.edge_w[base + lane] : 1.f;
        if (a.col_w) wv *= a.col_w[cidx];
      }
    }
    for (int j = 0; j < n; j += NS * UNROLL) {
      typename V::T v[UNROLL][VPL];
      float we[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int e = j + u * NS + slot;
        const int src = __shfl(cidx, e & 63, 64);
        we[u] = HAS_W ? __shfl(wv, e & 63, 64) : 1.f;
        const float* xr = a.x + (int64_t)src * d;
#pragma unroll
        for (int q = 0; q < VPL; ++q) {
          const int c = (q * LPR + sl) * W;
          // the dP score gather over a multi-GB user table streams its rows with nt loads (cfg4:
          // 32.4 -> 31.0 ms; on a table the Infinity Cache half holds, cfg3, 2.80 -> 3.42 ms, so
          // only above 1 GiB); the mean gathers keep the default policy (nt costs them 25-45 %:
          // the source-block passes and the Zipf-hot post rows live on cache reuse)
          if (SC && a.nt_load)
            v[u][q] = (e < n && c < d) ? V::load_nt(xr + c) : V::zero();
          else
            v[u][q] = (e < n && c < d) ? V::load(xr + c) : V::zero();
        }
      }
      if constexpr (SC) {
        const float cw = score == 1 ? *a.cscale * a.inv_e : a.inv_e;
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
          float sdot = 0.f;
#pragma unroll
          for (int q = 0; q < VPL; ++q) sdot += V::dot(rv[q], v[u][q]);
          sdot = slot_sum<LPR>(sdot);
          const float sg = sigmoid_t(sdot, exp_neg_abs(sdot));
          we[u] = cw * (score == 1 ? sg - 1.f : sg);
        }
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
#pragma unroll
        for (int q = 0; q < VPL; ++q) {
          if (HAS_W || SC) V::fma(acc[q], we[u], v[u][q]);
          else V::add(acc[q], v[u][q]);
        }
    }
  }
}

// combine the NS slots (lanes sl, sl+LPR, ...)
template <int LPR, int VPL, int W>
__device__ __forceinline__ void slot_combine(typename Vec<W>::T (&acc)[VPL]) {
  using V = Vec<W>;
#pragma unroll
  for (int m = LPR; m < 64; m <<= 1)
#pragma unroll
    for (int q = 0; q < VPL; ++q) V::add(acc[q], V::shfl_xor(acc[q], m));
}

// one item (a light row, or a chunk of a heavy row) per wave
template <int LPR, int VPL, int W, int UNROLL, bool HAS_W, bool SC>
__device__ __forceinline__ void gather_item(const GatherArgs& a, const int64_t item) {
  using V = Vec<W>;
  const int lane = threadIdx.x & 63;
  const int sl = lane % LPR;
  const bool writer = lane < LPR;
  int64_t row, beg, end;
  float* dst;
  bool partial;
  const bool two = SC && a.rowptr2;             // hgnn_score_gather2: + the negatives' segment
  bool own = true;                              // this wave sums the row's (first) segment
  if (item < a.n_rows) {                       // light row: whole row in this wave
    row = item;
    beg = a.rowptr[row];
    end = a.rowptr[row + 1];
    if (end - beg > a.chunk) {                  // heavy: handled by chunks + fixup ...
      if (!two) return;
      own = false;                              // ... the second list's segment still here
    }
    dst = a.out + row * a.d;
    partial = false;
  } else {                                      // chunk of a heavy row -> slab slot
    const int64_t slot = item - a.n_rows;
    int64_t lo = 0, hi = a.n_heavy;             // heavy_first[h] <= slot < heavy_first[h+1]
    while (hi - lo > 1) {
      int64_t mid = (lo + hi) >> 1;
      if (a.heavy_first[mid] <= slot) lo = mid; else hi = mid;
    }
    row = a.heavy_rows[lo];
    const int64_t k = slot - a.heavy_first[lo];
    beg = a.rowptr[row] + k * a.chunk;
    end = min<int64_t>(beg + a.chunk, a.rowptr[row + 1]);
    dst = a.slab + slot * a.d;
    partial = true;
  }
  typename V::T acc[VPL], rv[VPL];
#pragma unroll
  for (int q = 0; q < VPL; ++q) {
    acc[q] = V::zero();
    const int c = (q * LPR + sl) * W;
    rv[q] = (SC && c < a.d) ? V::load(a.rowvec + row * a.d + c) : V::zero();
  }
  if (own) segment_sum<LPR, VPL, W, UNROLL, HAS_W, SC>(a, a.col, a.score, beg, end, rv, acc);
  if (two && !partial)
    segment_sum<LPR, VPL, W, UNROLL, HAS_W, SC>(a, a.col2, 2, a.rowptr2[row], a.rowptr2[row + 1],
                                                rv, acc);
  slot_combine<LPR, VPL, W>(acc);
  if (!writer) return;
  float s = 1.f;
  if (!partial) {
    if (a.row_w) s = a.row_w[row];
    else if (a.mean) s = end > beg ? 1.f / (float)(end - beg) : 0.f;
  }
#pragma unroll
  for (int q = 0; q < VPL; ++q) {
    const int c = (q * LPR + sl) * W;
    if (c < a.d) {
      typename V::T r = acc[q];
      if (!partial) {
        V::scale(r, s);
        if (a.accumulate && (a.acc_limit == 0 || row < a.acc_limit)) V::add(r, V::load(dst + c));
      }
      if (a.nt_store) V::store_nt(dst + c, r);
      else V::store(dst + c, r);
    }
  }
}

template <int LPR, int VPL, int W, int UNROLL, bool HAS_W, bool SC = false>
__global__ void __launch_bounds__(256) k_gather(const GatherArgs a) {
  const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= a.n_items) return;
  gather_item<LPR, VPL, W, UNROLL, HAS_W, SC>(a, item);
}

// Several gathers of one row width in one launch (hgnn_gather_reduce_multi): job j owns the
// waves [base[j], base[j + 1]); light rows only (no heavy-row plan), distinct outputs.
constexpr int kGatherMultiMax = 8;
struct GatherMulti {
  GatherArgs j[kGatherMultiMax];
  int64_t base[kGatherMultiMax + 1];
  int32_t n;
};

template <int LPR, int VPL, int W, int UNROLL, bool HAS_W>
__global__ void __launch_bounds__(256) k_gather_multi(const GatherMulti m) {
  // the wave index made scalar: the job search and the job's arguments are then scalar loads
  // (a per-lane index fetched every argument with vector loads, one more dependent round trip
  // per wave — slower than the separate launches)
  const int64_t item = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (item >= m.base[m.n]) return;
  int j = 0;
  while (j + 1 < m.n && item >= m.base[j + 1]) ++j;
  gather_item<LPR, VPL, W, UNROLL, HAS_W, false>(m.j[j], item - m.base[j]);
}

// Heavy rows: out[row] (+)= s * sum_k slab[first + k].  One block per heavy row: S slices of
// the chunk list (strided) x the row's vectors, then a fixed-order LDS tree => deterministic.
template <int W>
__global__ void __launch_bounds__(256) k_fixup(const GatherArgs a) {
  using V = Vec<W>;
  __shared__ typename V::T buf[256];
  const int64_t h = blockIdx.x;
  const int64_t row = a.heavy_rows[h];
  const int64_t f0 = a.heavy_first[h], f1 = a.heavy_first[h + 1];
  const int64_t deg = a.rowptr[row + 1] - a.rowptr[row];
  const float s = a.row_w ? a.row_w[row] : (a.mean ? (deg > 0 ? 1.f / (float)deg : 0.f) : 1.f);
  const int nvec = (a.d + W - 1) / W;
  int cpb = 1;
  while (cpb < nvec && cpb < 256) cpb <<= 1;
  const int S = 256 / cpb;
  const int slice = threadIdx.x / cpb, cv = threadIdx.x % cpb;
  for (int c0 = 0; c0 < nvec; c0 += cpb) {
    const int c = (c0 + cv) * W;
    typename V::T r = V::zero();
    if (c < a.d) {
      int64_t k = f0 + slice;
      for (; k + 3 * S < f1; k += 4 * S) {   // 4 independent loads in flight
        typename V::T x0 = V::load(a.slab + k * a.d + c);
        typename V::T x1 = V::load(a.slab + (k + S) * a.d + c);
        typename V::T x2 = V::load(a.slab + (k + 2 * S) * a.d + c);
        typename V::T x3 = V::load(a.slab + (k + 3 * S) * a.d + c);
        V::add(x0, x1); V::add(x2, x3); V::add(x0, x2); V::add(r, x0);
      }
      for (; k < f1; k += S) V::add(r, V::load(a.slab + k * a.d + c));
    }
    buf[threadIdx.x] = r;
    __syncthreads();
    for (int st = S / 2; st >= 1; st >>= 1) {
      if (slice < st) {
        typename V::T t = buf[threadIdx.x];
        V::add(t, buf[threadIdx.x + st * cpb]);
        buf[threadIdx.x] = t;
      }
      __syncthreads();
    }
    if (slice == 0 && c < a.d) {
      typename V::T t = buf[threadIdx.x];
      V::scale(t, s);
      float* o = a.out + row * a.d + c;
      if (a.accumulate || a.rowptr2) V::add(t, V::load(o));
      V::store(o, t);
    }
    __syncthreads();
  }
}

template <int LPR, int VPL, int W, int UNROLL>
static int launch_gather(const GatherArgs& a, bool has_w, hipStream_t stream) {
  const dim3 grid((unsigned)cdiv(a.n_items, 4)), block(256);
  if (a.score)
    hipLaunchKernelGGL((k_gather<LPR, VPL, W, UNROLL, false, true>), grid, block, 0, stream, a);
  else if (has_w)
    hipLaunchKernelGGL((k_gather<LPR, VPL, W, UNROLL, true>), grid, block, 0, stream, a);
  else
    hipLaunchKernelGGL((k_gather<LPR, VPL, W, UNROLL, false>), grid, block, 0, stream, a);
  return check_launch("k_gather");
}

static int dispatch_gather(const GatherArgs& a, bool has_w, hipStream_t stream) {
  const int d = a.d;
  if (d % 4 == 0) {
    const int nv = d / 4;  // float4 vectors per row
    if (nv <= 4) return launch_gather<4, 1, 4, 4>(a, has_w, stream);
    if (nv <= 8) return launch_gather<8, 1, 4, 4>(a, has_w, stream);
    if (nv <= 16) {
      // d = 64: rows in flight per wave (4 x UNROLL) chosen per variant on cfg2 (MI355X).  The
      // mean gathers take 32: user rows average 20 edges, so one round of loads covers most of
      // them (user<-post 0.84 -> 0.80 ms); the weighted K2 24 (0.50 -> 0.485 ms); the score
      // gather keeps 16 (its dot products hold more registers: 1.39 ms at 16, 1.50 at 32).
      const dim3 grid((unsigned)cdiv(a.n_items, 4)), block(256);
      if (a.score)
        hipLaunchKernelGGL((k_gather<16, 1, 4, 4, false, true>), grid, block, 0, stream, a);
      else if (has_w)
        hipLaunchKernelGGL((k_gather<16, 1, 4, 6, true>), grid, block, 0, stream, a);
      else
        hipLaunchKernelGGL((k_gather<16, 1, 4, 8, false>), grid, block, 0, stream, a);
      return check_launch("k_gather");
    }
    // d = 128 (512-B rows): 8, 12 or 16 rows in flight measured the same on cfg3 and cfg4; 8
    // kept (the 12- and 16-deep forms are no longer built)
    if (nv <= 32) return launch_gather<32, 1, 4, 4>(a, has_w, stream);
    if (nv <= 64) return launch_gather<64, 1, 4, 4>(a, has_w, stream);
    if (nv <= 128) return launch_gather<64, 2, 4, 2>(a, has_w, stream);
    if (nv <= 256) return launch_gather<64, 4, 4, 2>(a, has_w, stream);
    return fail(HGNN_E_UNSUPPORTED, "gather: d=%d > 1024", d);
  }
  if (d <= 16) return launch_gather<16, 1, 1, 4>(a, has_w, stream);
  if (d <= 64) return launch_gather<64, 1, 1, 4>(a, has_w, stream);
  if (d <= 256) return launch_gather<64, 4, 1, 2>(a, has_w, stream);
  if (d <= 1024) return launch_gather<64, 16, 1, 1>(a, has_w, stream);
  return fail(HGNN_E_UNSUPPORTED, "gather: d=%d > 1024", d);
}

// nt above 1 GiB: cfg4's 4.6 GB user table and its 4.6 GB user-side outputs.  Output rows of
// the dP gather / K2s / means are read by another kernel long after they left L2 (cfg4 step
// 168.1 -> 167.5 ms with nt stores, mostly the dP gather); cfg2/cfg3 tables stay cache-resident.
constexpr int64_t kNtBytes = int64_t(1) << 30;
static void nt_policy(GatherArgs& a, int64_t n_x) {
  a.nt_load = a.score && n_x * a.d * 4 >= kNtBytes ? 1 : 0;
  a.nt_store = (a.score ? a.nt_load : a.n_rows * a.d * 4 >= kNtBytes) ? 1 : 0;
}

static int run_gather(GatherArgs a, hipStream_t stream) {
  if (a.d <= 0 || a.n_rows < 0 || a.n_heavy < 0 || a.chunk <= 0)
    return fail(HGNN_E_ARG, "gather: bad sizes d=%d n_rows=%lld chunk=%d", a.d,
                (long long)a.n_rows, a.chunk);
  if (a.n_rows == 0) return HGNN_OK;
  // x / col may be null only for a CSR without edges (nothing is dereferenced then)
  if (!a.rowptr || !a.out) return fail(HGNN_E_ARG, "gather: null rowptr/out");
  if (a.n_heavy > 0 && (!a.heavy_rows || !a.heavy_first || !a.slab))
    return fail(HGNN_E_ARG, "gather: heavy rows without plan/slab");
  const bool has_w = a.edge_w || a.col_w;
  if (a.score && (has_w || a.mean || !a.rowvec || (a.score == 1 && !a.cscale)))
    return fail(HGNN_E_ARG, "score_gather: bad mode/arguments");
  if (a.rowptr2 && a.score != 1)
    return fail(HGNN_E_ARG, "score_gather2: needs mode 1 for the first list");
  if (int rc = dispatch_gather(a, has_w, stream)) return rc;
  if (a.n_heavy > 0) {
    const dim3 grid((unsigned)a.n_heavy), block(256);
    if (a.d % 4 == 0) hipLaunchKernelGGL(k_fixup<4>, grid, block, 0, stream, a);
    else hipLaunchKernelGGL(k_fixup<1>, grid, block, 0, stream, a);
    return check_launch("k_fixup");
  }
  return HGNN_OK;
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_gather_reduce(const float* x, int64_t n_x, int32_t d, const int32_t* rowptr,
                       const int32_t* col, int64_t n_rows, const float* edge_w,
                       const float* col_w, int32_t flags, const int32_t* heavy_rows,
                       const int32_t* heavy_first, int64_t n_heavy, int64_t n_chunks,
                       int32_t chunk, float* slab, float* out, hgnn_stream_t stream) {
  GatherArgs a{};
  a.x = x; a.rowptr = rowptr; a.col = col; a.edge_w = edge_w; a.col_w = col_w;
  a.heavy_rows = heavy_rows; a.heavy_first = heavy_first; a.slab = slab; a.out = out;
  a.n_rows = n_rows; a.n_heavy = n_heavy; a.n_items = n_rows + (n_heavy > 0 ? n_chunks : 0);
  a.d = d; a.chunk = chunk; a.mean = (flags & HGNN_MEAN) ? 1 : 0;
  a.accumulate = (flags & HGNN_ACCUMULATE) ? 1 : 0;
  nt_policy(a, n_x);
  return run_gather(a, as_stream(stream));
}

int hgnn_gather_reduce_multi(int32_t n_jobs, const float* const* x, const int64_t* n_x, int32_t d,
                             const int32_t* const* rowptr, const int32_t* const* col,
                             const int64_t* n_rows, const float* const* edge_w, int32_t flags,
                             const int64_t* acc_limit, float* const* out,
                             hgnn_stream_t stream_) {
  if (n_jobs < 1 || n_jobs > kGatherMultiMax || d <= 0 || d % 4 || d > 512)
    return fail(HGNN_E_ARG, "gather_reduce_multi: n_jobs=%d (1..%d) d=%d (4..512, % 4)", n_jobs,
                kGatherMultiMax, d);
  GatherMulti m{};
  m.n = n_jobs;
  bool has_w = false;
  for (int j = 0; j < n_jobs; ++j) {
    GatherArgs& a = m.j[j];
    if (n_rows[j] < 0 || (n_rows[j] > 0 && (!rowptr[j] || !out[j])))
      return fail(HGNN_E_ARG, "gather_reduce_multi: job %d: null rowptr/out", j);
    for (int i = 0; i < j; ++i)
      if (n_rows[j] > 0 && out[i] == out[j])
        return fail(HGNN_E_ARG, "gather_reduce_multi: jobs %d and %d share an output", i, j);
    a.x = x[j]; a.rowptr = rowptr[j]; a.col = col[j]; a.out = out[j];
    a.edge_w = edge_w ? edge_w[j] : nullptr;
    has_w |= a.edge_w != nullptr;
    a.n_rows = n_rows[j]; a.n_items = n_rows[j]; a.d = d; a.chunk = INT32_MAX;
    a.mean = (flags & HGNN_MEAN) ? 1 : 0;
    a.accumulate = (flags & HGNN_ACCUMULATE) ? 1 : 0;
    a.acc_limit = acc_limit ? acc_limit[j] : 0;
    if (a.acc_limit < 0) return fail(HGNN_E_ARG, "gather_reduce_multi: acc_limit[%d] < 0", j);
    nt_policy(a, n_x[j]);
    m.base[j + 1] = m.base[j] + n_rows[j];
  }
  if (m.base[n_jobs] == 0) return HGNN_OK;
  const dim3 grid((unsigned)cdiv(m.base[n_jobs], 4)), block(256);
  hipStream_t stream = as_stream(stream_);
  // the row widths dispatch_gather takes at d % 4 == 0 (d = 64: its mean / weighted depths)
  const int nv = d / 4;
#define HGNN_GM(LPR, VPL, U, UW)                                                                 \
  if (has_w) hipLaunchKernelGGL((k_gather_multi<LPR, VPL, 4, UW, true>), grid, block, 0, stream, m); \
  else hipLaunchKernelGGL((k_gather_multi<LPR, VPL, 4, U, false>), grid, block, 0, stream, m);
  if (nv <= 4) { HGNN_GM(4, 1, 4, 4) }
  else if (nv <= 8) { HGNN_GM(8, 1, 4, 4) }
  else if (nv <= 16) { HGNN_GM(16, 1, 8, 6) }
  else if (nv <= 32) { HGNN_GM(32, 1, 4, 4) }
  else if (nv <= 64) { HGNN_GM(64, 1, 4, 4) }
  else { HGNN_GM(64, 2, 2, 2) }
#undef HGNN_GM
  return check_launch("k_gather_multi");
}

int hgnn_gather_reduce_scaled(const float* x, int64_t n_x, int32_t d, const int32_t* rowptr,
                              const int32_t* col, int64_t n_rows, const float* edge_w,
                              const float* col_w, const float* row_w, int32_t flags,
                              const int32_t* heavy_rows, const int32_t* heavy_first,
                              int64_t n_heavy, int64_t n_chunks, int32_t chunk, float* slab,
                              float* out, hgnn_stream_t stream) {
  if (row_w && (flags & HGNN_MEAN))
    return fail(HGNN_E_ARG, "gather_reduce_scaled: row_w replaces HGNN_MEAN, not both");
  GatherArgs a{};
  a.x = x; a.rowptr = rowptr; a.col = col; a.edge_w = edge_w; a.col_w = col_w; a.row_w = row_w;
  a.heavy_rows = heavy_rows; a.heavy_first = heavy_first; a.slab = slab; a.out = out;
  a.n_rows = n_rows; a.n_heavy = n_heavy; a.n_items = n_rows + (n_heavy > 0 ? n_chunks : 0);
  a.d = d; a.chunk = chunk; a.mean = 0;
  a.accumulate = (flags & HGNN_ACCUMULATE) ? 1 : 0;
  nt_policy(a, n_x);
  return run_gather(a, as_stream(stream));
}

int hgnn_gather_mean_fwd(const float* x_src, int64_t n_src, int32_t d, const int32_t* rowptr,
                         const int32_t* col, int64_t n_dst, const int32_t* heavy_rows,
                         const int32_t* heavy_first, int64_t n_heavy, int64_t n_chunks,
                         int32_t chunk, float* slab, float* aggr, hgnn_stream_t stream) {
  return hgnn_gather_reduce(x_src, n_src, d, rowptr, col, n_dst, nullptr, nullptr, HGNN_MEAN,
                            heavy_rows, heavy_first, n_heavy, n_chunks, chunk, slab, aggr,
                            stream);
}

int hgnn_scatter_mean_bwd(const float* grad_aggr, int64_t n_dst, const float* inv_deg,
                          const int32_t* t_rowptr, const int32_t* t_col, int64_t n_src,
                          int32_t d, const int32_t* heavy_rows, const int32_t* heavy_first,
                          int64_t n_heavy, int64_t n_chunks, int32_t chunk, float* slab,
                          float* grad_x_src, int32_t accumulate, hgnn_stream_t stream) {
  if (!inv_deg && n_src > 0) return fail(HGNN_E_ARG, "scatter_mean_bwd: inv_deg is null");
  return hgnn_gather_reduce(grad_aggr, n_dst, d, t_rowptr, t_col, n_src, nullptr, inv_deg,
                            accumulate ? HGNN_ACCUMULATE : 0, heavy_rows, heavy_first, n_heavy,
                            n_chunks, chunk, slab, grad_x_src, stream);
}

int hgnn_score_gather(const float* x, int64_t n_x, const float* rowvec, int32_t d,
                      const int32_t* rowptr, const int32_t* col, int64_t n_rows, int32_t mode,
                      const float* cscale, float inv_e, const int32_t* heavy_rows,
                      const int32_t* heavy_first, int64_t n_heavy, int64_t n_chunks,
                      int32_t chunk, float* slab, float* out, int32_t accumulate,
                      hgnn_stream_t stream) {
  if (mode != 1 && mode != 2) return fail(HGNN_E_ARG, "score_gather: mode=%d", mode);
  GatherArgs a{};
  a.x = x; a.rowptr = rowptr; a.col = col;
  a.heavy_rows = heavy_rows; a.heavy_first = heavy_first; a.slab = slab; a.out = out;
  a.n_rows = n_rows; a.n_heavy = n_heavy; a.n_items = n_rows + (n_heavy > 0 ? n_chunks : 0);
  a.d = d; a.chunk = chunk; a.accumulate = accumulate ? 1 : 0;
  a.rowvec = rowvec; a.cscale = cscale; a.inv_e = inv_e; a.score = mode;
  nt_policy(a, n_x);
  return run_gather(a, as_stream(stream));
}

int hgnn_score_gather2(const float* x, int64_t n_x, const float* rowvec, int32_t d,
                       const int32_t* rowptr, const int32_t* col, const int32_t* rowptr_n,
                       const int32_t* col_n, int64_t n_rows, const float* cscale, float inv_e,
                       const int32_t* heavy_rows, const int32_t* heavy_first, int64_t n_heavy,
                       int64_t n_chunks, int32_t chunk, float* slab, float* out,
                       hgnn_stream_t stream) {
  if (!rowptr_n && n_rows > 0) return fail(HGNN_E_ARG, "score_gather2: rowptr_n is null");
  GatherArgs a{};
  a.x = x; a.rowptr = rowptr; a.col = col;
  a.heavy_rows = heavy_rows; a.heavy_first = heavy_first; a.slab = slab; a.out = out;
  a.n_rows = n_rows; a.n_heavy = n_heavy; a.n_items = n_rows + (n_heavy > 0 ? n_chunks : 0);
  a.d = d; a.chunk = chunk;
  a.rowvec = rowvec; a.cscale = cscale; a.inv_e = inv_e; a.score = 1;
  a.rowptr2 = rowptr_n; a.col2 = col_n;
  nt_policy(a, n_x);
  return run_gather(a, as_stream(stream));
}

}  // extern "C"
