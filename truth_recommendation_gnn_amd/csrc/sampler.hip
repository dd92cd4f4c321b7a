// Neighbour sampling for mini-batch training (BASELINE cfg5: fanout [15, 10], 4 relations).
//
// The reference trains full-batch (train_gnn.py:254) and has no sampler; SURVEY.md §8 f4 asks for
// one so the 10M-node / 4-relation config runs on mini-batches.  Semantics follow the usual
// layer-wise scheme (PyG NeighborLoader, replace=False): for every destination node of a layer
// and every relation into its type, keep all in-neighbours if there are at most `fanout`, else a
// uniform sample of `fanout` distinct neighbour positions (duplicate edges are distinct positions).
//
//   k_sample_count  counts[i] = min(deg(dst_i), fanout)          (fanout < 0: all neighbours)
//   (exclusive scan -> the block's rowptr)
//   k_sample_fill   one wave per destination: Floyd's k-of-n without replacement, the chosen
//                   positions held one per lane ("already taken?" is one ballot); the random
//                   draws come from a counter-based hash of (seed, global dst id, draw index), so
//                   a node's sample does not depend on which batch it sits in, and runs repeat
//   relabel         the next layer's node set: the current destination nodes first (their order
//                   kept, so the root term is a prefix view), then every newly reached node in
//                   order of first appearance among the sampled items (PyG's order) — a hash set
//                   over the ids of this call (O(items) work, independent of the graph's node
//                   count), atomicMin for the first appearance and one exclusive scan, so the
//                   result is deterministic.
#include "sampler_common.h"

namespace hgnn {

__global__ void k_sample_count(const int32_t* rowptr, int64_t n_rows, const int32_t* dst_ids,
                               int64_t n, int32_t fanout, int32_t* counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  counts[i] = sample_count(rowptr, n_rows, dst_ids[i], fanout);
}

__global__ void __launch_bounds__(256) k_sample_fill(const int32_t* rowptr, const int32_t* col,
                                                     int64_t n_rows, const int32_t* dst_ids,
                                                     int64_t n, int32_t fanout, uint64_t seed,
                                                     const int32_t* out_rowptr,
                                                     int32_t* out_col) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= n) return;
  sample_fill<64>(rowptr, col, n_rows, dst_ids[w], fanout, seed, out_col + out_rowptr[w]);
}

// ---- one hop over every relation into the frontier: one launch per phase ------------------------
// Destinations of all relations concatenated (relation r owns [off[r], off[r+1])); the counts are
// scanned once over the concatenation and split back into zero-based per-relation rowptrs.
struct HopTab {
  const int32_t* rowptr[kHopMax];
  const int32_t* col[kHopMax];
  const int32_t* dst[kHopMax];
  int32_t* out_rowptr[kHopMax];
  int32_t* out_col[kHopMax];
  int64_t n_rows[kHopMax];
  int64_t off[kHopMax + 1];
  int32_t n_rel;
  int32_t fanout;
  uint64_t seed;
};

__device__ __forceinline__ int hop_rel(const HopTab& t, int64_t i) {
  int r = 0;
  while (r + 1 < t.n_rel && i >= t.off[r + 1]) ++r;
  return r;
}

__global__ void k_hop_count(const HopTab t, int32_t* counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.off[t.n_rel]) return;
  const int r = hop_rel(t, i);
  counts[i] = sample_count(t.rowptr[r], t.n_rows[r], t.dst[r][i - t.off[r]], t.fanout);
}

// entry j <= n_r of relation r sits at g = off[r] + r + j
__global__ void k_hop_rowptr(const HopTab t, const int32_t* pre, int32_t* totals) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= t.off[t.n_rel] + t.n_rel) return;
  int r = 0;
  while (r + 1 < t.n_rel && g >= t.off[r + 1] + r + 1) ++r;
  const int64_t j = g - t.off[r] - r;
  const int32_t v = pre[t.off[r] + j] - pre[t.off[r]];
  t.out_rowptr[r][j] = v;
  if (j == t.off[r + 1] - t.off[r]) totals[r] = v;
}

// G lanes per destination (16 when the fanout fits: 4 destinations per wave)
template <int G>
__global__ void __launch_bounds__(256) k_hop_fill(const HopTab t) {
  const int64_t w = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / G) +
                    (threadIdx.x & 63) / G;
  if (w >= t.off[t.n_rel]) return;
  const int r = hop_rel(t, w);
  const int64_t j = w - t.off[r];
  sample_fill<G>(t.rowptr[r], t.col[r], t.n_rows[r], t.dst[r][j], t.fanout, t.seed,
                 t.out_col[r] + t.out_rowptr[r][j]);
}

// ---- relabel: a hash set over the ids this call sees, O(n_prefix + n_items) work --------------
// One call relabels every node type of a hop: the table is keyed by id * T + type, the items of
// the types lie in consecutive ranges of one buffer, and the new ids of a type are ranked by one
// exclusive scan over all items (a type's ranks start at the scan's value at its first item).
// slot arrays (capacity a power of two >= 2·(n_prefix + n_items)): key (-1 empty), ppos (prefix
// position or -1), first (smallest item position of a non-prefix id; atomicMin, so deterministic)
constexpr int kRelabelMaxTypes = 8;
struct RelabelTab {
  int32_t* key;
  int32_t* ppos;
  int32_t* first;
  int32_t* nflags;   // per type: ~flags of the prefix check (all ones from the key memset)
  uint32_t mask;
  int shift;   // 64 - log2(capacity)
  int32_t T;   // node types
  const int32_t* prefix[kRelabelMaxTypes];
  int32_t* nodes[kRelabelMaxTypes];
  int64_t id_limit[kRelabelMaxTypes];   // prefix ids must lie in [0, id_limit) (< 0: no limit)
  int64_t p_off[kRelabelMaxTypes + 1];  // concatenated prefix positions per type
  int64_t i_off[kRelabelMaxTypes + 1];  // item ranges per type
};

__device__ __forceinline__ int rl_type(const int64_t* off, int T, int64_t i) {
  int t = 0;
  while (t + 1 < T && i >= off[t + 1]) ++t;
  return t;
}

// Prefix ids (the previous frontier, or the seeds) are expected distinct and in range: with the
// check on, a repeated id (found already inserted) clears bit 0 of its type's nflags word, an id
// outside [0, id_limit) bit 1 (that id is not inserted) — read back with the node counts.
__global__ void k_relabel_prefix(RelabelTab t) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= t.p_off[t.T]) return;
  const int ty = rl_type(t.p_off, t.T, g);
  const int64_t i = g - t.p_off[ty];
  const int32_t id = t.prefix[ty][i];
  t.nodes[ty][i] = id;
  if (id < 0 || (t.id_limit[ty] >= 0 && id >= t.id_limit[ty])) {   // flagged, never inserted
    if (t.nflags) atomicAnd(&t.nflags[ty], ~2);
    return;
  }
  bool found = false;
  const uint32_t s = rl_find_or_insert(t.key, t.mask, t.shift, id * t.T + ty, &found);
  if (found && t.nflags) atomicAnd(&t.nflags[ty], ~1);
  t.ppos[s] = (int32_t)i;   // one writer per slot when the prefix ids are distinct
}

__global__ void k_relabel_insert(RelabelTab t, const int32_t* items, int32_t* slot_of) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= t.i_off[t.T]) return;
  const int ty = rl_type(t.i_off, t.T, k);
  const uint32_t s = rl_find_or_insert(t.key, t.mask, t.shift, items[k] * t.T + ty);
  slot_of[k] = (int32_t)s;
  if (t.ppos[s] < 0) atomicMin(&t.first[s], (int32_t)k);
}

__global__ void k_relabel_flags(RelabelTab t, const int32_t* slot_of, int32_t* flags) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= t.i_off[t.T]) return;
  const int32_t s = slot_of[k];
  flags[k] = t.ppos[s] < 0 && t.first[s] == (int32_t)k;
}

__global__ void k_relabel_assign(RelabelTab t, const int32_t* items, const int32_t* slot_of,
                                 const int32_t* rank, int32_t* local) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= t.i_off[t.T]) return;
  const int ty = rl_type(t.i_off, t.T, k);
  const int32_t s = slot_of[k];
  const int32_t pp = t.ppos[s];
  if (pp >= 0) {
    local[k] = pp;
    return;
  }
  const int32_t f = t.first[s];
  const int64_t n_prefix = t.p_off[ty + 1] - t.p_off[ty];
  const int32_t l = (int32_t)(n_prefix + rank[f] - rank[t.i_off[ty]]);
  local[k] = l;
  if (f == (int32_t)k) t.nodes[ty][l] = items[k];
}

__global__ void k_relabel_count(RelabelTab t, const int32_t* rank, int32_t* d_count2) {
  const int ty = threadIdx.x;
  if (ty >= t.T) return;
  const int64_t n_new = t.i_off[t.T] > 0 ? rank[t.i_off[ty + 1]] - rank[t.i_off[ty]] : 0;
  // checked calls return (count, flags) per type; the plain single-type call only the count
  const int stride = t.nflags ? 2 : 1;
  d_count2[stride * ty] = (int32_t)(t.p_off[ty + 1] - t.p_off[ty] + n_new);
  if (t.nflags) d_count2[2 * ty + 1] = ~t.nflags[ty];
}

static size_t relabel_ws(int64_t n_prefix, int64_t n_items, size_t* scan_b) {
  const int64_t cap = relabel_cap(n_prefix + n_items);
  exclusive_scan_i32(nullptr, nullptr, n_items < 1 ? 1 : n_items, nullptr, scan_b, 0);
  return 3 * align_up((size_t)cap * 4, 256) + 256 + 3 * align_up((size_t)(n_items + 1) * 4, 256) +
         *scan_b + 256;
}

}  // namespace hgnn

using namespace hgnn;

static int relabel(int32_t T, const int32_t* const* prefix, const int64_t* n_prefix,
                   const int64_t* id_limit, const int32_t* items, const int64_t* n_items,
                   int32_t* local_out, int32_t* const* nodes_out, int32_t* d_count, bool check,
                   void* ws, size_t ws_bytes, hipStream_t stream);

extern "C" {

int hgnn_sample_neighbors(const int32_t* rowptr, const int32_t* col, int64_t n_rows,
                          const int32_t* dst_ids, int64_t n_dst, int32_t fanout, uint64_t seed,
                          int32_t* out_rowptr, int32_t* out_col, void* ws, size_t ws_bytes,
                          hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_rows < 0 || n_dst < 0 || fanout == 0 || fanout > 64)
    return fail(HGNN_E_ARG, "sample_neighbors: n_rows=%lld n_dst=%lld fanout=%d (1..64 or <0)",
                (long long)n_rows, (long long)n_dst, fanout);
  if (!out_rowptr || (n_dst > 0 && (!rowptr || !dst_ids)))
    return fail(HGNN_E_ARG, "sample_neighbors: null pointer");
  if (n_dst == 0) {
    (void)hipMemsetAsync(out_rowptr, 0, sizeof(int32_t), stream);
    return check_launch("sample_neighbors(empty)");
  }
  size_t scan_b = 0;
  exclusive_scan_i32(nullptr, nullptr, n_dst, nullptr, &scan_b, stream);
  const size_t need = align_up((size_t)n_dst * 4, 256) + scan_b;
  if (ws_bytes < need) return fail(HGNN_E_WS, "sample_neighbors: workspace too small");
  Workspace w(ws, ws_bytes);
  int32_t* counts = w.take<int32_t>(n_dst);
  void* scan_ws = w.take<char>(scan_b);
  hipLaunchKernelGGL(k_sample_count, dim3((unsigned)cdiv(n_dst, 256)), dim3(256), 0, stream,
                     rowptr, n_rows, dst_ids, n_dst, fanout, counts);
  if (int rc = check_launch("k_sample_count")) return rc;
  if (int rc = exclusive_scan_i32(counts, out_rowptr, n_dst, scan_ws, &scan_b, stream)) return rc;
  if (!out_col) return HGNN_OK;   // count-only call
  return hgnn_sample_fill(rowptr, col, n_rows, dst_ids, n_dst, fanout, seed, out_rowptr, out_col,
                          stream_);
}

int hgnn_sample_fill(const int32_t* rowptr, const int32_t* col, int64_t n_rows,
                     const int32_t* dst_ids, int64_t n_dst, int32_t fanout, uint64_t seed,
                     const int32_t* out_rowptr, int32_t* out_col, hgnn_stream_t stream) {
  if (n_rows < 0 || n_dst < 0 || fanout == 0 || fanout > 64)
    return fail(HGNN_E_ARG, "sample_fill: n_rows=%lld n_dst=%lld fanout=%d (1..64 or <0)",
                (long long)n_rows, (long long)n_dst, fanout);
  if (n_dst == 0) return HGNN_OK;
  if (!rowptr || !dst_ids || !out_rowptr || !out_col)
    return fail(HGNN_E_ARG, "sample_fill: null pointer");
  hipLaunchKernelGGL(k_sample_fill, dim3((unsigned)cdiv(n_dst, 4)), dim3(256), 0,
                     as_stream(stream), rowptr, col, n_rows, dst_ids, n_dst, fanout, seed,
                     out_rowptr, out_col);
  return check_launch("k_sample_fill");
}

static int hop_table(HopTab& t, int32_t n_rel, const int32_t* const* rowptrs,
                     const int32_t* const* cols, const int64_t* n_rows,
                     const int32_t* const* dst_ids, const int64_t* n_dst, int32_t fanout,
                     const char* what) {
  if (n_rel < 1 || n_rel > kHopMax || fanout == 0 || fanout > 64 || !rowptrs || !n_rows ||
      !dst_ids || !n_dst)
    return fail(HGNN_E_ARG, "%s: n_rel=%d (1..%d) fanout=%d (1..64 or <0)", what, n_rel, kHopMax,
                fanout);
  t.n_rel = n_rel;
  t.fanout = fanout;
  t.off[0] = 0;
  for (int r = 0; r < n_rel; ++r) {
    if (n_rows[r] < 0 || n_dst[r] < 0 || (n_dst[r] > 0 && (!rowptrs[r] || !dst_ids[r])))
      return fail(HGNN_E_ARG, "%s: relation %d", what, r);
    t.rowptr[r] = rowptrs[r];
    t.col[r] = cols ? cols[r] : nullptr;
    t.dst[r] = dst_ids[r];
    t.n_rows[r] = n_rows[r];
    t.off[r + 1] = t.off[r] + n_dst[r];
  }
  if (t.off[n_rel] >= (int64_t)INT32_MAX) return fail(HGNN_E_ARG, "%s: too many destinations", what);
  return HGNN_OK;
}

size_t hgnn_sample_hop_ws_bytes(int64_t n_total_dst) {
  const int64_t n = n_total_dst < 1 ? 1 : n_total_dst;
  size_t scan_b = 0;
  exclusive_scan_i32(nullptr, nullptr, n, nullptr, &scan_b, 0);
  return 2 * align_up((size_t)(n + 1) * 4, 256) + scan_b + 256;
}

int hgnn_sample_hop_count(int32_t n_rel, const int32_t* const* rowptrs, const int64_t* n_rows,
                          const int32_t* const* dst_ids, const int64_t* n_dst, int32_t fanout,
                          int32_t* const* out_rowptrs, int32_t* d_totals, void* ws,
                          size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  HopTab t{};
  if (int rc = hop_table(t, n_rel, rowptrs, nullptr, n_rows, dst_ids, n_dst, fanout,
                         "sample_hop_count"))
    return rc;
  if (!out_rowptrs || !d_totals) return fail(HGNN_E_ARG, "sample_hop_count: null output");
  for (int r = 0; r < n_rel; ++r) {
    if (!out_rowptrs[r]) return fail(HGNN_E_ARG, "sample_hop_count: out_rowptrs[%d] is null", r);
    t.out_rowptr[r] = out_rowptrs[r];
  }
  const int64_t n = t.off[n_rel];
  if (ws_bytes < hgnn_sample_hop_ws_bytes(n))
    return fail(HGNN_E_WS, "sample_hop_count: workspace too small");
  Workspace w(ws, ws_bytes);
  int32_t* counts = w.take<int32_t>(n + 1);
  int32_t* pre = w.take<int32_t>(n + 1);
  size_t scan_b = 0;
  exclusive_scan_i32(nullptr, nullptr, n < 1 ? 1 : n, nullptr, &scan_b, stream);
  void* scan_ws = w.take<char>(scan_b);
  if (n > 0) {
    hipLaunchKernelGGL(k_hop_count, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, t,
                       counts);
    if (int rc = check_launch("k_hop_count")) return rc;
  }
  if (int rc = exclusive_scan_i32(counts, pre, n, scan_ws, &scan_b, stream)) return rc;
  hipLaunchKernelGGL(k_hop_rowptr, dim3((unsigned)cdiv(n + n_rel, 256)), dim3(256), 0, stream, t,
                     pre, d_totals);
  return check_launch("k_hop_rowptr");
}

int hgnn_sample_hop_fill(int32_t n_rel, const int32_t* const* rowptrs, const int32_t* const* cols,
                         const int64_t* n_rows, const int32_t* const* dst_ids,
                         const int64_t* n_dst, int32_t fanout, uint64_t seed,
                         const int32_t* const* out_rowptrs, int32_t* const* out_cols,
                         hgnn_stream_t stream_) {
  HopTab t{};
  if (int rc = hop_table(t, n_rel, rowptrs, cols, n_rows, dst_ids, n_dst, fanout,
                         "sample_hop_fill"))
    return rc;
  if (!out_rowptrs || !out_cols || !cols) return fail(HGNN_E_ARG, "sample_hop_fill: null array");
  for (int r = 0; r < n_rel; ++r) {
    if (n_dst[r] > 0 && (!cols[r] || !out_rowptrs[r] || !out_cols[r]))
      return fail(HGNN_E_ARG, "sample_hop_fill: relation %d: null pointer", r);
    t.out_rowptr[r] = const_cast<int32_t*>(out_rowptrs[r]);
    t.out_col[r] = out_cols[r];
  }
  t.seed = seed;
  const int64_t n = t.off[n_rel];
  if (n == 0) return HGNN_OK;
  if (fanout > 0 && fanout <= 16)
    hipLaunchKernelGGL(k_hop_fill<16>, dim3((unsigned)cdiv(n, 16)), dim3(256), 0,
                       as_stream(stream_), t);
  else
    hipLaunchKernelGGL(k_hop_fill<64>, dim3((unsigned)cdiv(n, 4)), dim3(256), 0,
                       as_stream(stream_), t);
  return check_launch("k_hop_fill");
}

size_t hgnn_sample_ws_bytes(int64_t n_dst) {
  size_t scan_b = 0;
  exclusive_scan_i32(nullptr, nullptr, n_dst < 1 ? 1 : n_dst, nullptr, &scan_b, 0);
  return align_up((size_t)(n_dst < 1 ? 1 : n_dst) * 4, 256) + scan_b + 256;
}

size_t hgnn_relabel_ws_bytes(int64_t n_prefix, int64_t n_items) {
  size_t scan_b = 0;
  return relabel_ws(n_prefix < 0 ? 0 : n_prefix, n_items < 0 ? 0 : n_items, &scan_b);
}

int hgnn_relabel(const int32_t* prefix, int64_t n_prefix, const int32_t* items, int64_t n_items,
                 int32_t* local_out, int32_t* nodes_out, int32_t* d_count, void* ws,
                 size_t ws_bytes, hgnn_stream_t stream_) {
  int32_t* nodes[1] = {nodes_out};
  const int64_t no_limit = -1;   // unchecked: a limit of 0 would flag every id (an empty type)
  return relabel(1, &prefix, &n_prefix, &no_limit, items, &n_items, local_out, nodes, d_count, false,
                 ws, ws_bytes, as_stream(stream_));
}

int hgnn_relabel_checked(const int32_t* prefix, int64_t n_prefix, int64_t id_limit,
                         const int32_t* items, int64_t n_items, int32_t* local_out,
                         int32_t* nodes_out, int32_t* d_count2, void* ws, size_t ws_bytes,
                         hgnn_stream_t stream_) {
  int32_t* nodes[1] = {nodes_out};
  return relabel(1, &prefix, &n_prefix, &id_limit, items, &n_items, local_out, nodes, d_count2,
                 true, ws, ws_bytes, as_stream(stream_));
}

size_t hgnn_relabel_multi_ws_bytes(int64_t n_prefix_total, int64_t n_items_total) {
  size_t scan_b = 0;
  return relabel_ws(n_prefix_total < 0 ? 0 : n_prefix_total,
                    n_items_total < 0 ? 0 : n_items_total, &scan_b);
}

int hgnn_relabel_multi(int32_t n_types, const int32_t* const* prefix, const int64_t* n_prefix,
                       const int64_t* id_limit, const int32_t* items, const int64_t* n_items,
                       int32_t* local_out, int32_t* const* nodes_out, int32_t* d_count2,
                       int32_t check, void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  return relabel(n_types, prefix, n_prefix, id_limit, items, n_items, local_out, nodes_out,
                 d_count2, check != 0, ws, ws_bytes, as_stream(stream_));
}


// ------------------------------------------------------------ static-capacity blocks (graphs)
// hgnn_pad_csr_multi: item i copies a sampled block relation's CSR (rowptr over n_dst rows,
// col[E]) into capacity buffers of d_cap + 1 / e_cap entries.  The e_cap - E padding entries
// point at sources dummy .. dummy + spread - 1 in turn (padded source rows: spread over many, so
// the transposed grouping the backward builds has no long padded row — one source row holding
// every padding entry made its K2 wave 0.5 ms) and are spread over the padded rows
// n_dst .. d_cap - 1 (row n_dst + j
// gets positions E + j (e_cap - E) / P .. E + (j + 1) (e_cap - E) / P, P = d_cap - n_dst), so the
// result is a valid CSR of exactly d_cap rows and e_cap entries whose real rows are untouched and
// no padded row is long.  With `map`, real entries become map[col] (local -> global ids).  An
// item with d_cap < 0 copies (and maps) col only: a node-id list padded with `dummy`.
constexpr int kPadMaxItems = 16;
struct PadItems {
  const int32_t* rowptr[kPadMaxItems];
  const int32_t* col[kPadMaxItems];
  const int32_t* map[kPadMaxItems];
  int32_t* rowptr_out[kPadMaxItems];
  int32_t* col_out[kPadMaxItems];
  int64_t n_dst[kPadMaxItems], e[kPadMaxItems], d_cap[kPadMaxItems], e_cap[kPadMaxItems];
  int32_t dummy[kPadMaxItems], spread[kPadMaxItems];
};

__global__ void __launch_bounds__(256) k_pad_csr(const PadItems a) {
  const int it = blockIdx.y;
  const int64_t n_dst = a.n_dst[it], E = a.e[it], D = a.d_cap[it], EC = a.e_cap[it];
  const int64_t span = (D + 1 > EC ? D + 1 : EC);
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < span;
       idx += (int64_t)gridDim.x * 256) {
    if (D >= 0 && idx <= D)
      a.rowptr_out[it][idx] = idx <= n_dst ? a.rowptr[it][idx]
                                           : (int32_t)(E + (idx - n_dst) * (EC - E) / (D - n_dst));
    if (idx < EC) {
      int32_t v = a.dummy[it] + (int32_t)((idx - E) % a.spread[it]);
      if (idx < E) {
        v = a.col[it][idx];
        if (a.map[it]) v = a.map[it][v];
      }
      a.col_out[it][idx] = v;
    }
  }
}

int hgnn_pad_csr_multi(int32_t n_items, const int32_t* const* rowptr, const int32_t* const* col,
                       const int32_t* const* map, const int64_t* n_dst, const int64_t* e,
                       int32_t* const* rowptr_out, int32_t* const* col_out, const int64_t* d_cap,
                       const int64_t* e_cap, const int32_t* dummy, const int32_t* spread,
                       hgnn_stream_t stream_) {
  if (n_items < 1 || n_items > kPadMaxItems)
    return fail(HGNN_E_ARG, "pad_csr_multi: n_items=%d (1..%d)", n_items, kPadMaxItems);
  PadItems a{};
  int64_t span = 1;
  for (int i = 0; i < n_items; ++i) {
    const bool csr = d_cap[i] >= 0;
    if (e[i] < 0 || e[i] > e_cap[i] || (e[i] > 0 && !col[i]) || !col_out[i] ||
        (csr && (n_dst[i] < 0 || n_dst[i] >= d_cap[i] || !rowptr[i] || !rowptr_out[i])) ||
        (!csr && e_cap[i] < 1) || (csr && e_cap[i] > e[i] && d_cap[i] <= n_dst[i]) ||
        e_cap[i] >= INT32_MAX || (spread && spread[i] < 1))
      return fail(HGNN_E_ARG,
                  "pad_csr_multi: item %d: n_dst=%lld E=%lld into capacity %lld rows / %lld "
                  "entries (a sampled block larger than its static capacity, or no padded row)",
                  i, (long long)n_dst[i], (long long)e[i], (long long)d_cap[i],
                  (long long)e_cap[i]);
    a.rowptr[i] = rowptr[i];
    a.col[i] = col[i];
    a.map[i] = map ? map[i] : nullptr;
    a.rowptr_out[i] = rowptr_out[i];
    a.col_out[i] = col_out[i];
    a.n_dst[i] = n_dst[i];
    a.e[i] = e[i];
    a.d_cap[i] = d_cap[i];
    a.e_cap[i] = e_cap[i];
    a.dummy[i] = dummy[i];
    a.spread[i] = spread ? spread[i] : 1;
    span = std::max<int64_t>(span, std::max<int64_t>(d_cap[i] + 1, e_cap[i]));
  }
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(span, 256), 1024);
  hipLaunchKernelGGL(k_pad_csr, dim3(gx, (unsigned)n_items), dim3(256), 0, as_stream(stream_), a);
  return check_launch("k_pad_csr");
}

// hgnn_gather_rows_multi: item i's rows out[i][r] = src[i][ids[i][r]] (d floats, r < n_rows[i])
// in one launch — the static step's root rows, gathered from the feature tables with the staged
// batch (minibatch.StaticBlocks.prepare).  One float4 per thread over the items' rows numbered
// consecutively; ids are not validated (the sampler's global ids, padded with 0).
constexpr int kGatherRowsMax = 8;
struct RowGather {
  const float4* src[kGatherRowsMax];
  const int32_t* ids[kGatherRowsMax];
  float4* out[kGatherRowsMax];
  int64_t base[kGatherRowsMax + 1];
  int32_t n_items, d4;
};

__global__ void __launch_bounds__(256) k_gather_rows(const RowGather g) {
  const int64_t total = g.base[g.n_items] * g.d4;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int64_t row = idx / g.d4;
    const int64_t c = idx - row * g.d4;
    int it = 0;
    while (it + 1 < g.n_items && row >= g.base[it + 1]) ++it;
    const int64_t r = row - g.base[it];
    g.out[it][r * g.d4 + c] = g.src[it][(int64_t)g.ids[it][r] * g.d4 + c];
  }
}

int hgnn_gather_rows_multi(int32_t n_items, const float* const* src, const int32_t* const* ids,
                           const int64_t* n_rows, int64_t d, float* const* out,
                           hgnn_stream_t stream_) {
  if (n_items < 1 || n_items > kGatherRowsMax || d < 4 || d % 4 || d / 4 > INT32_MAX)
    return fail(HGNN_E_ARG, "gather_rows_multi: n_items=%d (1..%d), d=%lld (a multiple of 4)",
                n_items, kGatherRowsMax, (long long)d);
  RowGather g{};
  g.n_items = n_items;
  g.d4 = (int32_t)(d / 4);
  for (int i = 0; i < n_items; ++i) {
    if (n_rows[i] < 0 || (n_rows[i] > 0 && (!src[i] || !ids[i] || !out[i])) ||
        ((uintptr_t)src[i] | (uintptr_t)out[i]) % 16)
      return fail(HGNN_E_ARG, "gather_rows_multi: item %d: null or unaligned rows", i);
    g.src[i] = reinterpret_cast<const float4*>(src[i]);
    g.ids[i] = ids[i];
    g.out[i] = reinterpret_cast<float4*>(out[i]);
    g.base[i + 1] = g.base[i] + n_rows[i];
  }
  const int64_t total = g.base[n_items] * g.d4;
  if (total == 0) return HGNN_OK;
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(total, 256), 8192);
  hipLaunchKernelGGL(k_gather_rows, dim3(gx), dim3(256), 0, as_stream(stream_), g);
  return check_launch("k_gather_rows");
}

}  // extern "C"

static int relabel(int32_t T, const int32_t* const* prefix, const int64_t* n_prefix,
                   const int64_t* id_limit, const int32_t* items, const int64_t* n_items,
                   int32_t* local_out, int32_t* const* nodes_out, int32_t* d_count, bool check,
                   void* ws, size_t ws_bytes, hipStream_t stream) {
  if (T < 1 || T > kRelabelMaxTypes || !prefix || !n_prefix || !id_limit || !n_items ||
      !nodes_out || !d_count)
    return fail(HGNN_E_ARG, "relabel: n_types=%d (1..%d) or null array", T, kRelabelMaxTypes);
  RelabelTab t{};
  t.T = T;
  t.p_off[0] = t.i_off[0] = 0;
  int64_t max_limit = 0;
  for (int ty = 0; ty < T; ++ty) {
    if (n_prefix[ty] < 0 || n_items[ty] < 0) return fail(HGNN_E_ARG, "relabel: bad sizes");
    if ((n_prefix[ty] > 0 && !prefix[ty]) || (n_prefix[ty] + n_items[ty] > 0 && !nodes_out[ty]))
      return fail(HGNN_E_ARG, "relabel: type %d: null pointer", ty);
    t.prefix[ty] = prefix[ty];
    t.nodes[ty] = nodes_out[ty];
    t.id_limit[ty] = id_limit[ty];
    max_limit = std::max<int64_t>(max_limit, id_limit[ty]);
    t.p_off[ty + 1] = t.p_off[ty] + n_prefix[ty];
    t.i_off[ty + 1] = t.i_off[ty] + n_items[ty];
  }
  const int64_t np = t.p_off[T], ni = t.i_off[T];
  if (np + ni >= (int64_t)INT32_MAX / 2) return fail(HGNN_E_ARG, "relabel: bad sizes");
  if (T > 1 && (max_limit <= 0 || max_limit * T >= (int64_t)INT32_MAX))
    return fail(HGNN_E_ARG, "relabel: %d types need id limits with limit x types < 2^31", T);
  if (ni > 0 && (!items || !local_out)) return fail(HGNN_E_ARG, "relabel: null items/local");
  size_t scan_b = 0;
  if (ws_bytes < relabel_ws(np, ni, &scan_b))
    return fail(HGNN_E_WS, "relabel: workspace too small");
  const int64_t cap = relabel_cap(np + ni);
  int log2cap = 0;
  while ((int64_t(1) << log2cap) < cap) ++log2cap;
  Workspace w(ws, ws_bytes);
  t.key = w.take<int32_t>(2 * cap + 64);   // key, ppos and the flag words: one 0xFF memset
  t.ppos = t.key + cap;
  t.nflags = check ? t.key + 2 * cap : nullptr;
  t.first = w.take<int32_t>(cap);
  t.mask = (uint32_t)(cap - 1);
  t.shift = 64 - log2cap;
  int32_t* slot_of = w.take<int32_t>(ni + 1);
  int32_t* flags = w.take<int32_t>(ni + 1);
  int32_t* rank = w.take<int32_t>(ni + 1);
  void* scan_ws = w.take<char>(scan_b);
  (void)hipMemsetAsync(t.key, 0xFF, (size_t)cap * 8 + 4 * kRelabelMaxTypes, stream);
  (void)hipMemsetAsync(t.first, 0x7F, (size_t)cap * 4, stream);     // "infinity"
  if (np > 0)
    hipLaunchKernelGGL(k_relabel_prefix, dim3((unsigned)cdiv(np, 256)), dim3(256), 0, stream, t);
  if (ni > 0) {
    const unsigned g = (unsigned)cdiv(ni, 256);
    hipLaunchKernelGGL(k_relabel_insert, dim3(g), dim3(256), 0, stream, t, items, slot_of);
    hipLaunchKernelGGL(k_relabel_flags, dim3(g), dim3(256), 0, stream, t, slot_of, flags);
    if (int rc = check_launch("k_relabel_flags")) return rc;
    if (int rc = exclusive_scan_i32(flags, rank, ni, scan_ws, &scan_b, stream)) return rc;
    hipLaunchKernelGGL(k_relabel_assign, dim3(g), dim3(256), 0, stream, t, items, slot_of, rank,
                       local_out);
  }
  hipLaunchKernelGGL(k_relabel_count, dim3(1), dim3(64), 0, stream, t, rank, d_count);
  return check_launch("relabel");
}
