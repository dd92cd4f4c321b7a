// Sync-free sampling of link mini-batches straight into static-capacity buffers (BASELINE cfg5;
// minibatch.StaticSampler).  The eager sampler (sampler.hip) sizes every launch on the host and
// reads the sizes back twice per hop; with a graph-replayed step that makes the host loop the
// bound (round 6: 1.05 ms of host time per batch, most of it waiting in those read-backs).  Here
// every count stays on the device: launches cover the static capacities (minibatch.capacities)
// and read the real counts from device memory, so a batch is queued without a single sync.
// Results are bit-identical to the eager sampler followed by hgnn_pad_csr_multi (tested):
//
//   hgnn_link_seeds        a link batch's seeds = the distinct endpoints, sorted, and every
//                          pair's local ids (torch.unique + searchsorted of minibatch.link_batch):
//                          one workgroup per node type sorts its keys in LDS (bitonic), ranks the
//                          distinct ones with one block scan and scatters the ranks back
//   hgnn_sample_hop_static one hop (count, scan, rowptr + padding, fill) over the frontier's
//                          capacity, each relation's real destination count read on the device
//   hgnn_relabel_static    the next frontier (hgnn_relabel_multi's order: prefix first, then new
//                          ids by first appearance) over capacity-laid-out items, the valid ones
//                          per relation read on the device; local ids written per relation
#include "sampler_common.h"

#include <algorithm>

namespace hgnn {

// ---------------------------------------------------------------------------- link seeds
constexpr int kSeedMax = 4096;   // keys per node type (2 x the positives for the post side)

__device__ __forceinline__ bool seed_less(int32_t ka, int32_t ia, int32_t kb, int32_t ib) {
  return ka < kb || (ka == kb && ia < ib);
}

// block 0: the users of the B positives; block 1: their posts, then the B negatives
__global__ void __launch_bounds__(1024) k_link_seeds(const int64_t* src, const int64_t* dst,
                                                     const int64_t* eid, const int64_t* neg,
                                                     int64_t B, int32_t* seeds_u,
                                                     int32_t* seeds_p, int32_t* pu, int32_t* pp,
                                                     int32_t* pn, int32_t* d_counts) {
  __shared__ int32_t skey[kSeedMax], sidx[kSeedMax];
  __shared__ int32_t wsum[16];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int n = (int)(b == 0 ? B : 2 * B);
  int P = 1;
  while (P < n) P <<= 1;
  for (int i = tid; i < P; i += 1024) {
    int32_t k = INT32_MAX;
    if (i < n) {
      if (b == 0) k = (int32_t)src[eid[i]];
      else k = (int32_t)(i < B ? dst[eid[i]] : neg[i - B]);
    }
    skey[i] = k;
    sidx[i] = i < n ? i : INT32_MAX;
  }
  __syncthreads();
  // bitonic sort of (key, index) ascending
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P; i += 1024) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const int32_t ki = skey[i], kj = skey[j], ii = sidx[i], ij = sidx[j];
          if (seed_less(kj, ij, ki, ii) == up) {
            skey[i] = kj; skey[j] = ki;
            sidx[i] = ij; sidx[j] = ii;
          }
        }
      }
      __syncthreads();
    }
  }
  // rank of the distinct keys: each thread scans PER = P / 1024 (<= 4) consecutive entries
  const int PER = P >= 1024 ? P / 1024 : 1;
  const int j0 = tid * PER;
  int f[4] = {0, 0, 0, 0}, s = 0;
  for (int q = 0; q < PER; ++q) {
    const int j = j0 + q;
    f[q] = j < n && (j == 0 || skey[j] != skey[j - 1]);
    s += f[q];
  }
  // inclusive scan of s over the block: wave shuffles, then the 16 wave totals
  const int lane = tid & 63, wv = tid >> 6;
  int x = s;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  int before = 0;
  for (int w = 0; w < wv; ++w) before += wsum[w];
  int r = before + x - s;   // distinct keys before this thread's first entry
  for (int q = 0; q < PER; ++q) {
    const int j = j0 + q;
    if (j >= n) break;
    r += f[q];
    const int u = r - 1;   // the rank of entry j's key
    const int32_t idx = sidx[j];
    if (b == 0) {
      if (f[q]) seeds_u[u] = skey[j];
      pu[idx] = u;
    } else {
      if (f[q]) seeds_p[u] = skey[j];
      if (idx < B) pp[idx] = u;
      else pn[idx - B] = u;
    }
  }
  if (tid == 1023) {
    int tot = 0;
    for (int w = 0; w < 16; ++w) tot += wsum[w];
    d_counts[b] = tot;
  }
}

// ---------------------------------------------------------------------------- one hop
// Relation r counts destinations [off[r], off[r] + cap[r]) of the concatenated capacity range;
// rows at or past its real count (*d_ndst[r], on the device) count 0.
struct SHop {
  const int32_t* rowptr[kHopMax];
  const int32_t* col[kHopMax];
  const int32_t* dst[kHopMax];
  const int32_t* d_ndst[kHopMax];
  int32_t* out_rowptr[kHopMax];   // cap + 1 entries: real rows, then the padded rows
  int32_t* fill[kHopMax];         // the sampled (global) source ids, CSR order
  int32_t* tail[kHopMax];         // the array whose padding entries [E, ecap) are written
  int64_t n_rows[kHopMax], cap[kHopMax], ecap[kHopMax];
  int64_t off[kHopMax + 1];
  int32_t dummy[kHopMax], spread[kHopMax];
  int32_t* d_E;                   // out: sampled entries per relation
  int32_t n_rel, fanout;
  uint64_t seed;
};

__device__ __forceinline__ int shop_rel(const SHop& t, int64_t i) {
  int r = 0;
  while (r + 1 < t.n_rel && i >= t.off[r + 1]) ++r;
  return r;
}

__global__ void k_shop_count(const SHop t, int32_t* counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.off[t.n_rel]) return;
  const int r = shop_rel(t, i);
  const int64_t j = i - t.off[r];
  counts[i] = j < *t.d_ndst[r]
                  ? sample_count(t.rowptr[r], t.n_rows[r], t.dst[r][j], t.fanout) : 0;
}

// rowptr over all cap + 1 rows (the real rows from the scan, the padded rows as
// hgnn_pad_csr_multi spreads them) and the padding entries of the tail array
__global__ void __launch_bounds__(256) k_shop_rowptr(const SHop t, const int32_t* pre) {
  const int r = blockIdx.y;
  const int64_t n = *t.d_ndst[r], D = t.cap[r], EC = t.ecap[r];
  const int32_t base = pre[t.off[r]];
  const int64_t E = pre[t.off[r] + n] - base;
  if (blockIdx.x == 0 && threadIdx.x == 0) t.d_E[r] = (int32_t)E;
  const int64_t span = D + 1 > EC ? D + 1 : EC;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < span;
       idx += (int64_t)gridDim.x * 256) {
    if (idx <= D)
      t.out_rowptr[r][idx] = idx <= n ? pre[t.off[r] + idx] - base
                                      : (int32_t)(E + (idx - n) * (EC - E) / (D - n));
    if (idx >= E && idx < EC) t.tail[r][idx] = t.dummy[r] + (int32_t)((idx - E) % t.spread[r]);
  }
}

template <int G>   // lanes per destination, as k_hop_fill
__global__ void __launch_bounds__(256) k_shop_fill(const SHop t) {
  const int64_t w = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / G) +
                    (threadIdx.x & 63) / G;
  if (w >= t.off[t.n_rel]) return;
  const int r = shop_rel(t, w);
  const int64_t j = w - t.off[r];
  if (j >= *t.d_ndst[r]) return;
  sample_fill<G>(t.rowptr[r], t.col[r], t.n_rows[r], t.dst[r][j], t.fanout, t.seed,
                 t.fill[r] + t.out_rowptr[r][j]);
}

// ---------------------------------------------------------------------------- relabel
// The eager relabel over capacity layouts: type ty's prefix holds *d_np[ty] ids of cap p_cap;
// item relation q owns slots [ibase[q], ibase[q + 1]) of which the first d_E[q] are valid;
// relations are grouped by their source type, types ascending, so type ty's items are
// the slots [i_off[ty], i_off[ty + 1]) and invalid slots rank as nothing.
struct SRelabel {
  int32_t* key;
  int32_t* ppos;
  int32_t* first;
  uint32_t mask;
  int shift;
  int32_t T, n_irel;
  const int32_t* prefix[kHopMax];
  const int32_t* d_np[kHopMax];
  int32_t* nodes[kHopMax];
  int64_t p_off[kHopMax + 1];
  int64_t i_off[kHopMax + 1];
  int64_t ibase[kHopMax + 1];
  int32_t irel_type[kHopMax];
  int32_t* local[kHopMax];
  const int32_t* d_E;
  int32_t* d_count;
};

__device__ __forceinline__ int srl_find(const int64_t* off, int n, int64_t i) {
  int t = 0;
  while (t + 1 < n && i >= off[t + 1]) ++t;
  return t;
}

__global__ void k_srl_prefix(const SRelabel t) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= t.p_off[t.T]) return;
  const int ty = srl_find(t.p_off, t.T, g);
  const int64_t i = g - t.p_off[ty];
  if (i >= *t.d_np[ty]) return;
  const int32_t id = t.prefix[ty][i];
  t.nodes[ty][i] = id;
  const uint32_t s = rl_find_or_insert(t.key, t.mask, t.shift, id * t.T + ty);
  t.ppos[s] = (int32_t)i;
}

__global__ void k_srl_insert(const SRelabel t, const int32_t* items, int32_t* slot_of) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= t.ibase[t.n_irel]) return;
  const int q = srl_find(t.ibase, t.n_irel, k);
  if (k - t.ibase[q] >= t.d_E[q]) {
    slot_of[k] = -1;
    return;
  }
  const uint32_t s = rl_find_or_insert(t.key, t.mask, t.shift, items[k] * t.T + t.irel_type[q]);
  slot_of[k] = (int32_t)s;
  if (t.ppos[s] < 0) atomicMin(&t.first[s], (int32_t)k);
}

__global__ void k_srl_flags(const SRelabel t, const int32_t* slot_of, int32_t* flags) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= t.ibase[t.n_irel]) return;
  const int32_t s = slot_of[k];
  flags[k] = s >= 0 && t.ppos[s] < 0 && t.first[s] == (int32_t)k;
}

__global__ void k_srl_assign(const SRelabel t, const int32_t* items, const int32_t* slot_of,
                             const int32_t* rank) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= t.ibase[t.n_irel]) return;
  const int32_t s = slot_of[k];
  if (s < 0) return;
  const int q = srl_find(t.ibase, t.n_irel, k);
  const int ty = t.irel_type[q];
  const int32_t pp = t.ppos[s];
  int32_t l = pp;
  if (pp < 0) {
    const int32_t f = t.first[s];
    l = *t.d_np[ty] + rank[f] - rank[t.i_off[ty]];
    if (f == (int32_t)k) t.nodes[ty][l] = items[k];
  }
  t.local[q][k - t.ibase[q]] = l;
}

__global__ void k_srl_count(const SRelabel t, const int32_t* rank) {
  const int ty = threadIdx.x;
  if (ty >= t.T) return;
  const int32_t n_new = t.ibase[t.n_irel] > 0 ? rank[t.i_off[ty + 1]] - rank[t.i_off[ty]] : 0;
  t.d_count[ty] = *t.d_np[ty] + n_new;
}

size_t srl_ws(int64_t np, int64_t ni, size_t* scan_b) {
  const int64_t cap = relabel_cap(np + ni);
  exclusive_scan_i32(nullptr, nullptr, ni < 1 ? 1 : ni, nullptr, scan_b, 0);
  return align_up((size_t)(2 * cap + 64) * 4, 256) + align_up((size_t)cap * 4, 256) +
         3 * align_up((size_t)(ni + 1) * 4, 256) + *scan_b + 256;
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_link_seeds(const int64_t* src, const int64_t* dst, const int64_t* edge_ids,
                    const int64_t* neg, int64_t B, int32_t* seeds_u, int32_t* seeds_p,
                    int32_t* pu, int32_t* pp, int32_t* pn, int32_t* d_counts,
                    hgnn_stream_t stream) {
  if (B < 1 || 2 * B > kSeedMax)
    return fail(HGNN_E_ARG, "link_seeds: B=%lld positives (1..%d)", (long long)B, kSeedMax / 2);
  if (!src || !dst || !edge_ids || !neg || !seeds_u || !seeds_p || !pu || !pp || !pn || !d_counts)
    return fail(HGNN_E_ARG, "link_seeds: null pointer");
  hipLaunchKernelGGL(k_link_seeds, dim3(2), dim3(1024), 0, as_stream(stream), src, dst, edge_ids,
                     neg, B, seeds_u, seeds_p, pu, pp, pn, d_counts);
  return check_launch("k_link_seeds");
}

int hgnn_sample_hop_static(int32_t n_rel, const int32_t* const* rowptrs,
                           const int32_t* const* cols, const int64_t* n_rows,
                           const int32_t* const* dst_ids, const int32_t* const* d_n_dst,
                           const int64_t* caps, const int64_t* ecaps, int32_t fanout,
                           uint64_t seed, int32_t* const* out_rowptrs, int32_t* const* fill_outs,
                           int32_t* const* tail_outs, const int32_t* dummy,
                           const int32_t* spread, int32_t* d_E, void* ws, size_t ws_bytes,
                           hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_rel < 1 || n_rel > kHopMax || fanout < 1 || fanout > 64 || !d_E)
    return fail(HGNN_E_ARG, "sample_hop_static: n_rel=%d (1..%d) fanout=%d (1..64)", n_rel,
                kHopMax, fanout);
  SHop t{};
  t.n_rel = n_rel;
  t.fanout = fanout;
  t.seed = seed;
  t.d_E = d_E;
  int64_t span = 1;
  for (int r = 0; r < n_rel; ++r) {
    // a static capacity holds every sample: ecap >= fanout x the real rows, cap > the real rows
    if (!rowptrs[r] || !cols[r] || !dst_ids[r] || !d_n_dst[r] || !out_rowptrs[r] ||
        !fill_outs[r] || !tail_outs[r] || caps[r] < 1 || ecaps[r] < 1 || spread[r] < 1 ||
        caps[r] >= INT32_MAX || ecaps[r] >= INT32_MAX)
      return fail(HGNN_E_ARG, "sample_hop_static: relation %d", r);
    t.rowptr[r] = rowptrs[r];
    t.col[r] = cols[r];
    t.n_rows[r] = n_rows[r];
    t.dst[r] = dst_ids[r];
    t.d_ndst[r] = d_n_dst[r];
    t.out_rowptr[r] = out_rowptrs[r];
    t.fill[r] = fill_outs[r];
    t.tail[r] = tail_outs[r];
    t.cap[r] = caps[r];
    t.ecap[r] = ecaps[r];
    t.dummy[r] = dummy[r];
    t.spread[r] = spread[r];
    t.off[r + 1] = t.off[r] + caps[r];
    span = std::max<int64_t>(span, std::max<int64_t>(caps[r] + 1, ecaps[r]));
  }
  const int64_t n = t.off[n_rel];
  if (n >= INT32_MAX) return fail(HGNN_E_ARG, "sample_hop_static: too many destinations");
  size_t scan_b = 0;
  exclusive_scan_i32(nullptr, nullptr, n, nullptr, &scan_b, stream);
  Workspace w(ws, ws_bytes);
  int32_t* counts = w.take<int32_t>(n + 1);
  int32_t* pre = w.take<int32_t>(n + 1);
  void* scan_ws = w.take<char>(scan_b);
  if (!counts || !pre || !scan_ws) return fail(HGNN_E_WS, "sample_hop_static: workspace too small");
  hipLaunchKernelGGL(k_shop_count, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, t, counts);
  if (int rc = check_launch("k_shop_count")) return rc;
  if (int rc = exclusive_scan_i32(counts, pre, n, scan_ws, &scan_b, stream)) return rc;
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(span, 256), 256);
  hipLaunchKernelGGL(k_shop_rowptr, dim3(gx, (unsigned)n_rel), dim3(256), 0, stream, t, pre);
  if (int rc = check_launch("k_shop_rowptr")) return rc;
  if (fanout <= 16)
    hipLaunchKernelGGL(k_shop_fill<16>, dim3((unsigned)cdiv(n, 16)), dim3(256), 0, stream, t);
  else
    hipLaunchKernelGGL(k_shop_fill<64>, dim3((unsigned)cdiv(n, 4)), dim3(256), 0, stream, t);
  return check_launch("k_shop_fill");
}

size_t hgnn_relabel_static_ws_bytes(int64_t prefix_cap_total, int64_t item_cap_total) {
  size_t scan_b = 0;
  return srl_ws(prefix_cap_total < 0 ? 0 : prefix_cap_total,
                item_cap_total < 0 ? 0 : item_cap_total, &scan_b);
}

int hgnn_relabel_static(int32_t n_types, const int32_t* const* prefix,
                        const int32_t* const* d_n_prefix, const int64_t* prefix_caps,
                        int32_t* const* nodes_out, const int64_t* nodes_caps, int32_t n_irel,
                        const int32_t* items, const int64_t* item_caps, const int32_t* irel_type,
                        const int32_t* d_E, int32_t* const* local_out, int32_t* d_count,
                        void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_types < 1 || n_types > kHopMax || n_irel < 0 || n_irel > kHopMax || !d_count ||
      (n_irel > 0 && (!items || !d_E)))
    return fail(HGNN_E_ARG, "relabel_static: n_types=%d n_irel=%d", n_types, n_irel);
  SRelabel t{};
  t.T = n_types;
  t.n_irel = n_irel;
  t.d_E = d_E;
  t.d_count = d_count;
  for (int ty = 0; ty < n_types; ++ty) {
    if (!prefix[ty] || !d_n_prefix[ty] || !nodes_out[ty] || prefix_caps[ty] < 0 ||
        nodes_caps[ty] < prefix_caps[ty])
      return fail(HGNN_E_ARG, "relabel_static: type %d", ty);
    t.prefix[ty] = prefix[ty];
    t.d_np[ty] = d_n_prefix[ty];
    t.nodes[ty] = nodes_out[ty];
    t.p_off[ty + 1] = t.p_off[ty] + prefix_caps[ty];
  }
  for (int q = 0; q < n_irel; ++q) {
    if (item_caps[q] < 0 || !local_out[q] || irel_type[q] < 0 || irel_type[q] >= n_types ||
        (q > 0 && irel_type[q] < irel_type[q - 1]))
      return fail(HGNN_E_ARG, "relabel_static: item relation %d (grouped by type, ascending)", q);
    t.local[q] = local_out[q];
    t.irel_type[q] = irel_type[q];
    t.ibase[q + 1] = t.ibase[q] + item_caps[q];
  }
  // type ty's items: from its first relation's base to the next type's
  for (int ty = 0, q = 0; ty <= n_types; ++ty) {
    while (q < n_irel && irel_type[q] < ty) ++q;
    t.i_off[ty] = q < n_irel ? t.ibase[q] : t.ibase[n_irel];
  }
  const int64_t np = t.p_off[n_types], ni = t.ibase[n_irel];
  if (np + ni >= (int64_t)INT32_MAX / 2) return fail(HGNN_E_ARG, "relabel_static: bad sizes");
  size_t scan_b = 0;
  if (ws_bytes < srl_ws(np, ni, &scan_b)) return fail(HGNN_E_WS, "relabel_static: workspace");
  const int64_t cap = relabel_cap(np + ni);
  int log2cap = 0;
  while ((int64_t(1) << log2cap) < cap) ++log2cap;
  Workspace w(ws, ws_bytes);
  t.key = w.take<int32_t>(2 * cap + 64);
  t.ppos = t.key + cap;
  t.first = w.take<int32_t>(cap);
  t.mask = (uint32_t)(cap - 1);
  t.shift = 64 - log2cap;
  int32_t* slot_of = w.take<int32_t>(ni + 1);
  int32_t* flags = w.take<int32_t>(ni + 1);
  int32_t* rank = w.take<int32_t>(ni + 1);
  void* scan_ws = w.take<char>(scan_b);
  (void)hipMemsetAsync(t.key, 0xFF, (size_t)cap * 8, stream);
  (void)hipMemsetAsync(t.first, 0x7F, (size_t)cap * 4, stream);   // "infinity"
  for (int ty = 0; ty < n_types; ++ty)   // node lists past their count read as id 0 (padding)
    (void)hipMemsetAsync(t.nodes[ty], 0, (size_t)nodes_caps[ty] * 4, stream);
  if (np > 0)
    hipLaunchKernelGGL(k_srl_prefix, dim3((unsigned)cdiv(np, 256)), dim3(256), 0, stream, t);
  if (ni > 0) {
    const unsigned g = (unsigned)cdiv(ni, 256);
    hipLaunchKernelGGL(k_srl_insert, dim3(g), dim3(256), 0, stream, t, items, slot_of);
    hipLaunchKernelGGL(k_srl_flags, dim3(g), dim3(256), 0, stream, t, slot_of, flags);
    if (int rc = check_launch("k_srl_flags")) return rc;
    if (int rc = exclusive_scan_i32(flags, rank, ni, scan_ws, &scan_b, stream)) return rc;
    hipLaunchKernelGGL(k_srl_assign, dim3(g), dim3(256), 0, stream, t, items, slot_of, rank);
  }
  hipLaunchKernelGGL(k_srl_count, dim3(1), dim3(64), 0, stream, t, rank);
  return check_launch("relabel_static");
}

}  // extern "C"
