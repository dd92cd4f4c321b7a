// Batched ranking metrics of the reference's evaluation (train_gnn.py:289-367), one wave per user.
//
// The reference scores each test user against the sorted set of test candidate posts, takes the
// top-K (torch.topk), and computes
//   Recall@K = |topK ∩ true| / len(true_posts)            (len counts duplicate test edges)
//   NDCG@K   = sklearn.metrics.ndcg_score(relevance, scores, k=K)   (binary relevance,
//              ignore_ties=False: tied scores share their group's mean gain)
// with one host round trip per user.  Here the scores of a batch of users come from one GEMM
// (the caller's [rows, n_cand] matrix) and this kernel does the rest for every row at once:
//   1. scan: the wave keeps ONE running top-(K+1) list, entry r on lane r (score desc, candidate
//      index asc).  Its last value is the exact entry threshold, so after a warm start (a bitonic
//      pick over the first chunk's lane maxima) almost every 2048-value stretch is rejected by a
//      single wave-uniform compare; the few survivors go in one at a time (ballot-popcount
//      position, shfl_up shift).  The list ends sorted, no merge needed, and its (K+1)-th entry
//      tells whether ties cross the cut;
//   2. recall: lane r binary-searches its winner in the row's sorted unique true candidates;
//   3. ties: sklearn's tie-averaged DCG (_tie_averaged_dcg) needs, for every distinct value among
//      the top K, how many entries of the whole row share it and how many of those are relevant.
//      When the best entry outside the top K is strictly below the K-th, every such group lies
//      inside the top K and the counts come from the list lanes; only a tie across the cut
//      costs a second scan of the row.  Then DCG / IDCG in float64.
// Deterministic: no atomics; ties in the top-K membership resolve to the lower candidate index.
#include "hgnn_common.h"

#include <float.h>

namespace hgnn {

struct TopkArgs {
  const float* scores;        // [n_rows][ld]
  int64_t ld;
  int64_t n_rows;
  int64_t n_cand;
  const int32_t* true_rowptr; // [n_rows+1] into true_cand
  const int32_t* true_cand;   // per row: sorted unique relevant candidate indices
  const int32_t* true_count;  // per row: number of test edges (duplicates counted)
  int32_t k;                  // min(K, n_cand)
  int32_t* topk_idx;          // [n_rows][k] or null
  double* recall;             // [n_rows]
  double* ndcg;               // [n_rows]
};

__device__ __forceinline__ bool better(float av, int ai, float bv, int bi) {
  return av > bv || (av == bv && ai < bi);
}

__device__ __forceinline__ bool in_sorted(const int32_t* p, int n, int x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (p[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo < n && p[lo] == x;
}

__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) x = fmaxf(x, __shfl_xor(x, m, 64));
  return x;
}

// x sorted descending across the 64 lanes (bitonic network on shuffles)
__device__ __forceinline__ float wave_sort_desc(float x, int lane) {
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
    for (int stride = size / 2; stride > 0; stride >>= 1) {
      const float y = __shfl_xor(x, stride, 64);
      const bool keep_max = ((lane & stride) == 0) == ((lane & size) == 0);
      x = keep_max ? fmaxf(x, y) : fminf(x, y);
    }
  return x;
}

// The wave's running top-L list, one entry per lane (lane r: the r-th best so far, by score desc
// then candidate index asc; lanes >= L hold nothing).  thr = the L-th best value (or a proven
// lower bound of the final one): anything strictly below it can never enter.
struct WaveTopL {
  float lv = -FLT_MAX;
  int li = INT_MAX;
  float thr = -FLT_MAX;
  int L;
  int lane;
  __device__ __forceinline__ void insert(float cs, int ci) {
    const bool mine_better = lane < L && better(lv, li, cs, ci);
    const int pos = __popcll(__ballot(mine_better));   // entries that stay ahead
    if (pos >= L) return;                              // wave-uniform
    const float uv = __shfl_up(lv, 1, 64);
    const int ui = __shfl_up(li, 1, 64);
    if (lane > pos && lane < L) { lv = uv; li = ui; }
    if (lane == pos) { lv = cs; li = ci; }
    thr = fmaxf(thr, __shfl(lv, L - 1, 64));
  }
  // all lanes call with their own (val, idx); candidates >= thr are inserted one at a time
  __device__ __forceinline__ void consider(float val, int idx) {
    unsigned long long cm = __ballot(val >= thr);
    while (cm) {
      const int src = __ffsll((long long)cm) - 1;
      insert(__shfl(val, src, 64), __shfl(idx, src, 64));
      cm = __ballot(val >= thr) & (~0ull << src << 1);   // lanes after src, re-filtered
    }
  }
};

__global__ void __launch_bounds__(256) k_topk_metrics(const TopkArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.n_rows) return;
  const float* sr = a.scores + row * a.ld;
  const int64_t C = a.n_cand;
  const int k = a.k;
  // 1. scan: the list tracks the top-(k+1) when there is a (k+1)-th entry (it tells whether ties
  //    cross the cut), else the top-k
  WaveTopL w;
  w.L = (C > k) ? k + 1 : k;
  w.lane = lane;
  const bool vec = (a.ld % 4 == 0) && (reinterpret_cast<uintptr_t>(a.scores) % 16 == 0);
  int64_t c0 = 0;
  if (vec) {
    constexpr int UN = 8;   // 8 float4 loads in flight per lane
    const int64_t C4 = C / 4 * 4;
    bool first = true;
    // wave-uniform trip count: the ballots below need every lane active
    for (int64_t cb = 0; cb < C4; cb += 256 * UN) {
      const int64_t c = cb + (int64_t)lane * 4;
      float4 s[UN];
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        const int64_t cu = c + u * 256;
        s[u] = cu < C4 ? *reinterpret_cast<const float4*>(sr + cu)
                       : make_float4(-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX);
      }
      float m = -FLT_MAX;
#pragma unroll
      for (int u = 0; u < UN; ++u) m = fmaxf(m, fmaxf(fmaxf(s[u].x, s[u].y), fmaxf(s[u].z, s[u].w)));
      if (first) {
        // warm start: the L-th largest of the 64 lane maxima is a lower bound of the final L-th
        // best (those maxima are L distinct entries of the row)
        w.thr = __shfl(wave_sort_desc(m, lane), w.L - 1, 64);
        first = false;
      }
      if (__ballot(m >= w.thr) == 0ull) continue;   // wave-uniform: nothing here can enter
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        const int cu = (int)(c + u * 256);
        w.consider(s[u].x, cu);
        w.consider(s[u].y, cu + 1);
        w.consider(s[u].z, cu + 2);
        w.consider(s[u].w, cu + 3);
      }
    }
    c0 = C4;
  }
  for (int64_t cb = c0; cb < C; cb += 64) {
    const int64_t c = cb + lane;
    w.consider(c < C ? sr[c] : -FLT_MAX, c < C ? (int)c : INT_MAX);
  }
  const float tv = lane < k ? w.lv : -FLT_MAX;
  const int ti = lane < k ? w.li : INT_MAX;
  const float vnext = (C > k) ? __shfl(w.lv, k, 64) : -FLT_MAX;
  if (a.topk_idx && lane < k) a.topk_idx[row * k + lane] = ti;
  // 3. recall
  const int32_t tb = a.true_rowptr[row], te = a.true_rowptr[row + 1];
  const int m_rel = te - tb;
  const int32_t* tc = a.true_cand + tb;
  const bool rel = lane < k && in_sorted(tc, m_rel, ti);
  const int hits = __popcll(__ballot(rel));
  // 4. tie groups among the top-k values: lane g < G holds group g's value, count and relevance
  const float prev = __shfl_up(tv, 1, 64);
  const bool first = lane < k && (lane == 0 || prev != tv);
  const unsigned long long firsts = __ballot(first);
  const int G = __popcll(firsts);
  // the value of group g sits on the lane of its g-th "first" flag
  float gval = -FLT_MAX;
  {
    unsigned long long f = firsts;
    for (int g = 0; g < G; ++g) {
      const int src = __ffsll((long long)f) - 1;
      const float val = __shfl(tv, src, 64);
      if (lane == g) gval = val;
      f &= f - 1;
    }
  }
  const float kth = __shfl(tv, k - 1, 64);   // the k-th value (ties may cross it)
  int gn = 0, gr = 0;
  if (!(C > k && vnext == kth)) {
    // no tie crosses the cut: every group lies inside the top-k lanes
    const unsigned long long relm = __ballot(rel);
    for (int g = 0; g < G; ++g) {
      const float gv = __shfl(gval, g, 64);
      const unsigned long long mem = __ballot(lane < k && tv == gv);
      if (lane == g) { gn = __popcll(mem); gr = __popcll(mem & relm); }
    }
  }
  for (int64_t base = 0; C > k && vnext == kth && base < C; base += 64) {
    const int64_t c = base + lane;
    const float s = c < C ? sr[c] : -FLT_MAX;
    unsigned long long hit = __ballot(c < C && s >= kth);
    while (hit) {   // rare: the top-k entries and their ties
      const int src = __ffsll((long long)hit) - 1;
      hit &= hit - 1;
      const float sv = __shfl(s, src, 64);
      const int cj = (int)(base + src);
      const unsigned long long gm = __ballot(lane < G && gval == sv);
      const int g = __ffsll((long long)gm) - 1;
      if (g >= 0 && lane == g) {
        ++gn;
        gr += in_sorted(tc, m_rel, cj) ? 1 : 0;
      }
    }
  }
  // group start ranks: exclusive prefix of gn over lanes 0..G-1
  int start = 0;
  {
    int inc = gn;   // inclusive scan of gn
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    start = inc - gn;
  }
  double dcg = 0.0;
  if (lane < G && gn > 0) {
    double dsum = 0.0;
    const int stop = min(start + gn, k);
    for (int rank = start; rank < stop; ++rank) dsum += 1.0 / log2((double)rank + 2.0);
    dcg = (double)gr / (double)gn * dsum;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) dcg += __shfl_xor(dcg, o, 64);
  if (lane == 0) {
    double idcg = 0.0;
    const int mi = min(k, m_rel);
    for (int i = 0; i < mi; ++i) idcg += 1.0 / log2((double)i + 2.0);
    const int cnt = a.true_count[row];
    a.recall[row] = cnt > 0 ? (double)hits / (double)cnt : 0.0;
    a.ndcg[row] = idcg > 0.0 ? dcg / idcg : 0.0;
  }
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_topk_metrics(const float* scores, int64_t n_rows, int64_t n_cand, int64_t ld,
                      const int32_t* true_rowptr, const int32_t* true_cand,
                      const int32_t* true_count, int32_t K, int32_t* topk_idx, double* recall,
                      double* ndcg, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_rows < 0 || n_cand < 0 || ld < n_cand || K < 1 || K > 63)
    return fail(HGNN_E_ARG, "topk_metrics: bad sizes rows=%lld cand=%lld ld=%lld K=%d",
                (long long)n_rows, (long long)n_cand, (long long)ld, K);
  if (n_rows == 0) return HGNN_OK;
  if (n_cand == 0 || n_cand >= INT_MAX)
    return fail(HGNN_E_ARG, "topk_metrics: n_cand=%lld", (long long)n_cand);
  if (!scores || !true_rowptr || !true_cand || !true_count || !recall || !ndcg)
    return fail(HGNN_E_ARG, "topk_metrics: null pointer");
  TopkArgs a{};
  a.scores = scores; a.ld = ld; a.n_rows = n_rows; a.n_cand = n_cand;
  a.true_rowptr = true_rowptr; a.true_cand = true_cand; a.true_count = true_count;
  a.k = (int32_t)(K < n_cand ? K : n_cand);
  a.topk_idx = topk_idx; a.recall = recall; a.ndcg = ndcg;
  const dim3 grid((unsigned)cdiv(n_rows, 4)), block(256);
  hipLaunchKernelGGL(k_topk_metrics, grid, block, 0, stream, a);
  return check_launch("k_topk_metrics");
}

}  // extern "C"
