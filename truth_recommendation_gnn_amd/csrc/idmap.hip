// Edge construction from raw ids on the device (the step before the path).
//
// The reference builds every edge list on the host, one DataFrame row at a time
// (build_edge_index_safe, train_gnn.py:40-73: three dict.get per row, rows with any unmapped id
// skipped; build_test_edges, test_gnn.py:34-55; the Series.map + dropna of build_graph.py:383-402).
// Here the id -> node-index dictionaries become open-addressing hash tables in HBM and the rows are
// mapped and compacted by three kernels:
//
//   k_idmap_insert   one thread per dictionary key: hash, then claim the first empty slot of its
//                    linear probe sequence with a 64-bit CAS on the slot's row field
//   k_idmap_lookup   one thread per query: hash, probe, and on a hash match compare the actual key
//                    (the integer, or the UTF-8 bytes), so a 64-bit hash collision can never turn
//                    a missing id into a hit — the result is exactly dict.get's
//   k_keep_flags / exclusive scan / k_compact
//                    keep the rows whose every column mapped, in row order (what the list appends
//                    of the reference loop produce)
//
// Keys are either integers (int64, the hash is the value) or strings in the Arrow layout (int64
// offsets + bytes; byte buffers readable 16 B past their last string).  A slot is {hash, key row}, 16 B, so one probe is one 16-B load; capacity is a
// power of two >= 2·n_keys, so the expected probe count stays below 2.  The table holds key rows,
// not values: lookups read vals[row] (8 B) after the match.
#include "hgnn_common.h"

namespace hgnn {

struct __align__(16) Slot {
  uint64_t hash;
  int64_t row;   // -1: empty
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// 8 bytes starting at p (any alignment) from three aligned dword loads; reads up to 11 bytes past
// p + 8, which the padding contract covers (Arrow pads its buffers to 64 B; the Python side adds
// 16 B).  Byte-wide loads were the first version: 2-3x slower on the 18-B ids of the bench.
__device__ __forceinline__ uint64_t load8(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const int sh = (int)(a & 3) * 8;
  const uint64_t lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  return sh ? (lo >> sh) | ((uint64_t)w[2] << (64 - sh)) : lo;
}

__device__ __forceinline__ uint64_t tail_mask(int64_t rem) {   // rem in [1, 8]
  return rem >= 8 ? ~0ull : ((1ull << (8 * rem)) - 1ull);
}

// 64-bit hash of a byte string: 8-byte little-endian words (the last one zero-padded) folded
// through a bijective mixer, the length folded in first (so "" and "\0" differ).
__device__ __forceinline__ uint64_t hash_bytes(const uint8_t* p, int64_t len) {
  uint64_t h = 0x243F6A8885A308D3ull ^ ((uint64_t)len * 0x9E3779B97F4A7C15ull);
  for (int64_t i = 0; i < len; i += 8) h = mix64(h ^ (load8(p + i) & tail_mask(len - i)));
  return mix64(h ^ 0x5851F42D4C957F2Dull);
}

__device__ __forceinline__ bool bytes_equal(const uint8_t* a, const uint8_t* b, int64_t len) {
  for (int64_t i = 0; i < len; i += 8)
    if ((load8(a + i) ^ load8(b + i)) & tail_mask(len - i)) return false;
  return true;
}

// slot index of a hash: the string hash is already mixed, the integer "hash" is the raw id
__device__ __forceinline__ uint64_t home(uint64_t h) { return mix64(h + 0x9E3779B97F4A7C15ull); }

__global__ void k_idmap_insert(const int64_t* key_ints, const int64_t* key_off,
                               const uint8_t* key_bytes, int64_t n, Slot* slots, uint64_t mask) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = key_ints ? (uint64_t)key_ints[i]
                              : hash_bytes(key_bytes + key_off[i], key_off[i + 1] - key_off[i]);
  uint64_t s = home(h) & mask;
  for (uint64_t probe = 0; probe <= mask; ++probe) {   // always ends: capacity >= 2 n
    auto* row = reinterpret_cast<unsigned long long*>(&slots[s].row);
    if (atomicCAS(row, ~0ull, (unsigned long long)i) == ~0ull) {
      slots[s].hash = h;   // read only by later launches
      return;
    }
    s = (s + 1) & mask;
  }
}

struct LookupArgs {
  const Slot* slots;
  uint64_t mask;
  const int64_t* key_off;    // string keys
  const uint8_t* key_bytes;
  const int64_t* vals;       // NULL: return the key row
  const int64_t* q_ints;
  const int64_t* q_off;
  const uint8_t* q_bytes;
  const uint8_t* q_valid;    // NULL: all valid
  int64_t n_q;
  int64_t* out;
};

__global__ void __launch_bounds__(256) k_idmap_lookup(LookupArgs a) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.n_q) return;
  int64_t res = -1;
  if (!a.q_valid || a.q_valid[q]) {
    const bool ints = a.q_ints != nullptr;
    const uint8_t* qp = nullptr;
    int64_t qlen = 0;
    uint64_t h;
    if (ints) {
      h = (uint64_t)a.q_ints[q];
    } else {
      qp = a.q_bytes + a.q_off[q];
      qlen = a.q_off[q + 1] - a.q_off[q];
      h = hash_bytes(qp, qlen);
    }
    uint64_t s = home(h) & a.mask;
    for (uint64_t probe = 0; probe <= a.mask; ++probe) {   // bounded even on a foreign table
      const Slot sl = a.slots[s];
      if (sl.row < 0) break;
      if (sl.hash == h) {
        bool eq = true;
        if (!ints) {
          const int64_t kb = a.key_off[sl.row], klen = a.key_off[sl.row + 1] - kb;
          eq = klen == qlen && bytes_equal(a.key_bytes + kb, qp, qlen);
        }
        if (eq) {
          res = a.vals ? a.vals[sl.row] : sl.row;
          break;
        }
      }
      s = (s + 1) & a.mask;
    }
  }
  a.out[q] = res;
}

constexpr int kMaxCols = 4;

struct CompactArgs {
  const int64_t* cols[kMaxCols];
  int64_t* outs[kMaxCols];
  int out_col[kMaxCols];
  int n_cols, n_outs;
  int64_t n;
};

__global__ void k_keep_flags(CompactArgs a, int32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  bool keep = true;
#pragma unroll
  for (int c = 0; c < kMaxCols; ++c)
    if (c < a.n_cols) keep &= a.cols[c][i] >= 0;
  flags[i] = keep;
}

__global__ void k_compact(CompactArgs a, const int32_t* flags, const int32_t* pos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n || !flags[i]) return;
  const int64_t p = pos[i];
#pragma unroll
  for (int o = 0; o < kMaxCols; ++o)
    if (o < a.n_outs) a.outs[o][p] = a.cols[a.out_col[o]][i];
}

__global__ void k_total(const int32_t* pos, int64_t n, int32_t* d_count) { *d_count = pos[n]; }

static size_t compact_ws(int64_t n, size_t* scan_b) {
  exclusive_scan_i32(nullptr, nullptr, n, nullptr, scan_b, 0);
  return 2 * align_up((size_t)(n + 1) * 4, 256) + *scan_b + 256;
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

int64_t hgnn_idmap_capacity(int64_t n_keys) {
  int64_t c = 16;
  while (c < 2 * n_keys) c <<= 1;
  return c;
}

int hgnn_idmap_build(const int64_t* key_ints, const int64_t* key_offsets, const uint8_t* key_bytes,
                     int64_t n_keys, void* slots, int64_t capacity, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_keys < 0 || capacity < 16 || (capacity & (capacity - 1)) || capacity < 2 * n_keys)
    return fail(HGNN_E_ARG, "idmap_build: n_keys=%lld capacity=%lld (power of two >= 2 n_keys)",
                (long long)n_keys, (long long)capacity);
  if (!slots || (n_keys > 0 && !key_ints && !(key_offsets && key_bytes)))
    return fail(HGNN_E_ARG, "idmap_build: null pointer");
  (void)hipMemsetAsync(slots, 0xFF, (size_t)capacity * sizeof(Slot), stream);
  if (n_keys > 0)
    hipLaunchKernelGGL(k_idmap_insert, dim3((unsigned)cdiv(n_keys, 256)), dim3(256), 0, stream,
                       key_ints, key_ints ? nullptr : key_offsets, key_bytes, n_keys,
                       static_cast<Slot*>(slots), (uint64_t)(capacity - 1));
  return check_launch("k_idmap_insert");
}

int hgnn_idmap_lookup(const void* slots, int64_t capacity, const int64_t* key_ints,
                      const int64_t* key_offsets, const uint8_t* key_bytes, const int64_t* vals,
                      const int64_t* q_ints, const int64_t* q_offsets, const uint8_t* q_bytes,
                      const uint8_t* q_valid, int64_t n_q, int64_t* out, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_q < 0 || capacity < 16 || (capacity & (capacity - 1)))
    return fail(HGNN_E_ARG, "idmap_lookup: n_q=%lld capacity=%lld", (long long)n_q,
                (long long)capacity);
  if (n_q == 0) return HGNN_OK;
  const bool ints = q_ints != nullptr;
  if (!slots || !out || (ints ? !key_ints : !(q_offsets && q_bytes && key_offsets && key_bytes)))
    return fail(HGNN_E_ARG, "idmap_lookup: null pointer (integer queries need integer keys, "
                            "string queries string keys)");
  LookupArgs a{static_cast<const Slot*>(slots), (uint64_t)(capacity - 1), key_offsets,
               key_bytes, vals, q_ints, q_offsets, q_bytes, q_valid, n_q, out};
  hipLaunchKernelGGL(k_idmap_lookup, dim3((unsigned)cdiv(n_q, 256)), dim3(256), 0, stream, a);
  return check_launch("k_idmap_lookup");
}

size_t hgnn_compact_rows_ws_bytes(int64_t n) {
  size_t scan_b = 0;
  return compact_ws(n < 1 ? 1 : n, &scan_b);
}

int hgnn_compact_rows(const int64_t* const* cols, int32_t n_cols, int64_t n,
                      int64_t* const* outs, const int32_t* out_col, int32_t n_outs,
                      int32_t* d_count, void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n < 0 || n >= (int64_t)INT32_MAX || n_cols < 1 || n_cols > kMaxCols || n_outs < 0 ||
      n_outs > kMaxCols)
    return fail(HGNN_E_ARG, "compact_rows: n=%lld n_cols=%d n_outs=%d", (long long)n, n_cols,
                n_outs);
  if (!cols || !d_count || (n_outs > 0 && (!outs || !out_col)))
    return fail(HGNN_E_ARG, "compact_rows: null pointer");
  CompactArgs a{};
  for (int c = 0; c < n_cols; ++c) {
    if (n > 0 && !cols[c]) return fail(HGNN_E_ARG, "compact_rows: column %d is null", c);
    a.cols[c] = cols[c];
  }
  for (int o = 0; o < n_outs; ++o) {
    if (out_col[o] < 0 || out_col[o] >= n_cols || (n > 0 && !outs[o]))
      return fail(HGNN_E_ARG, "compact_rows: output %d (column %d)", o, out_col[o]);
    a.outs[o] = outs[o];
    a.out_col[o] = out_col[o];
  }
  a.n_cols = n_cols;
  a.n_outs = n_outs;
  a.n = n;
  if (n == 0) {
    (void)hipMemsetAsync(d_count, 0, sizeof(int32_t), stream);
    return check_launch("compact_rows(empty)");
  }
  size_t scan_b = 0;
  if (ws_bytes < compact_ws(n, &scan_b)) return fail(HGNN_E_WS, "compact_rows: workspace too small");
  Workspace w(ws, ws_bytes);
  int32_t* flags = w.take<int32_t>(n + 1);
  int32_t* pos = w.take<int32_t>(n + 1);
  void* scan_ws = w.take<char>(scan_b);
  const unsigned grid = (unsigned)cdiv(n, 256);
  hipLaunchKernelGGL(k_keep_flags, dim3(grid), dim3(256), 0, stream, a, flags);
  if (int rc = check_launch("k_keep_flags")) return rc;
  if (int rc = exclusive_scan_i32(flags, pos, n, scan_ws, &scan_b, stream)) return rc;
  hipLaunchKernelGGL(k_total, dim3(1), dim3(1), 0, stream, pos, n, d_count);
  if (n_outs > 0)
    hipLaunchKernelGGL(k_compact, dim3(grid), dim3(256), 0, stream, a, flags, pos);
  return check_launch("k_compact");
}

}  // extern "C"
