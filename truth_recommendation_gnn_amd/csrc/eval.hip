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

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

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
  const int32_t* row_map;     // null, or: row r's true sets and outputs live at row_map[r]
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

// Recall and NDCG of one row from its top list (lane r < k: the r-th best, tv / ti; vnext: the
// (k+1)-th value, or -FLT_MAX when there is none).  sr: the row's scores, for the second scan when
// a tie crosses the cut; when sr is null that case writes nothing and returns false (the caller
// redoes the row from materialised scores).  tr: where the row's true sets and outputs live.
__device__ bool row_metrics(const TopkArgs& a, int64_t tr, int lane, int k, int64_t C, float tv,
                            int ti, float vnext, const float* sr) {
  const float kth = __shfl(tv, k - 1, 64);   // the k-th value (ties may cross it)
  if (C > k && vnext == kth && !sr) return false;
  // 3. recall
  const int32_t tb = a.true_rowptr[tr], te = a.true_rowptr[tr + 1];
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
    const int cnt = a.true_count[tr];
    a.recall[tr] = cnt > 0 ? (double)hits / (double)cnt : 0.0;
    a.ndcg[tr] = idcg > 0.0 ? dcg / idcg : 0.0;
  }
  return true;
}

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
  row_metrics(a, a.row_map ? a.row_map[row] : row, lane, k, C, tv, ti, vnext, sr);
}


// ---- fused scoring + top-L: the score matrix is never materialised ---------------------------
// One workgroup = 4 waves x 32 users; the candidates stream through LDS in chunks of TC rows
// (double-buffered, next chunk prefetched into registers during the MFMA work of the current one).
// Scores come from fp32 MFMA 16x16x4 with the candidates as the A operand (rows) and the users as
// B (columns), so each lane ends with 4 candidates x 1 user per 16x16 tile and compares them with
// ONE threshold, its user's current L-th value.  Candidates that pass go, one at a time, into the
// user's list in LDS (entry r on lane r: the same sorted-list insert as WaveTopL).  A 16x16 tile
// of scores costs D/4 MFMAs; the rejection test costs one max3 + one compare per lane.
constexpr int kStUsersPerWave = 32;
constexpr int kStWaves = 4;
constexpr int kStThreads = kStWaves * 64;

struct ScoreTopkArgs {
  const float* U;         // [n_u_rows][d] user embeddings
  const int32_t* rows;    // null, or the U row of each output row
  int64_t n_rows;
  const float* P;         // [>= n_cand][d] candidate embeddings
  int64_t n_cand;
  int32_t L;              // list length, 1..64
  float* topv;            // [n_rows][L] scores, best first
  int32_t* topi;          // [n_rows][L] candidate indices
};

template <int D>
struct StCfg {
  static constexpr int TC = 64;              // candidates per chunk
  static constexpr int S = D + 8;            // LDS row stride (dwords): b128 fragment reads
  static constexpr int KC = D / 16;          // float4 fragments per row per lane
  static constexpr int LOADS = TC * D / 4 / kStThreads;   // float4 per thread per chunk
};

__device__ __forceinline__ void st_insert(float* lvs, int* lis, int L, int lane, float cs, int ci,
                                          float& newthr) {
  const float v = lane < L ? lvs[lane] : -FLT_MAX;
  const int x = lane < L ? lis[lane] : INT_MAX;
  const bool mine_better = lane < L && better(v, x, cs, ci);
  const int pos = __popcll(__ballot(mine_better));
  newthr = -FLT_MAX;
  if (pos >= L) return;   // wave-uniform: equal score, higher index than the L-th entry
  const float uv = __shfl_up(v, 1, 64);
  const int ux = __shfl_up(x, 1, 64);
  if (lane > pos && lane < L) { lvs[lane] = uv; lis[lane] = ux; }
  if (lane == pos) { lvs[lane] = cs; lis[lane] = ci; }
  newthr = (pos == L - 1) ? cs : __shfl(v, L - 2 < 0 ? 0 : L - 2, 64);
}

template <int D>
__global__ void __launch_bounds__(kStThreads) k_score_topk(const ScoreTopkArgs a) {
  using Cfg = StCfg<D>;
  constexpr int TC = Cfg::TC, S = Cfg::S, KC = Cfg::KC, LOADS = Cfg::LOADS;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* cbuf = lds;                                   // [2][TC][S]
  float* lv_all = lds + 2 * TC * S;                    // [4 waves][32 users][L]
  const int L = a.L;
  int* li_all = reinterpret_cast<int*>(lv_all + kStWaves * kStUsersPerWave * L);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * (kStWaves * kStUsersPerWave) +
                       wave * kStUsersPerWave;
  float* lvw = lv_all + wave * kStUsersPerWave * L;
  int* liw = li_all + wave * kStUsersPerWave * L;
  for (int e = lane; e < kStUsersPerWave * L; e += 64) { lvw[e] = -FLT_MAX; liw[e] = INT_MAX; }
  // user fragments (B operand): lane (i, g) holds user i's columns 16c + 4g .. +3
  float4 uf[2][KC];
  float thr[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int64_t r = row0 + nt * 16 + i;
    const bool ok = r < a.n_rows;
    const int64_t ur = ok ? (a.rows ? (int64_t)a.rows[r] : r) : 0;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      uf[nt][c] = ok ? *reinterpret_cast<const float4*>(a.U + ur * D + c * 16 + 4 * g)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
    thr[nt] = ok ? -FLT_MAX : FLT_MAX;   // rows past the end never take anything
  }
  const int64_t C = a.n_cand;
  const int64_t n_chunks = (C + TC - 1) / TC;
  // chunk staging: thread t loads float4 number t + kStThreads q of the chunk (row-major TC x D)
  float4 nxt[LOADS];
  auto load_chunk = [&](int64_t ch) {
#pragma unroll
    for (int q = 0; q < LOADS; ++q) {
      const int f = threadIdx.x + kStThreads * q;
      const int rr = f / (D / 4), cc = (f % (D / 4)) * 4;
      const int64_t cand = ch * TC + rr;
      nxt[q] = cand < C ? *reinterpret_cast<const float4*>(a.P + cand * D + cc)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int q = 0; q < LOADS; ++q) {
      const int f = threadIdx.x + kStThreads * q;
      const int rr = f / (D / 4), cc = (f % (D / 4)) * 4;
      *reinterpret_cast<float4*>(cbuf + buf * TC * S + rr * S + cc) = nxt[q];
    }
  };
  load_chunk(0);
  store_chunk(0);
  __syncthreads();
  for (int64_t ch = 0; ch < n_chunks; ++ch) {
    const int buf = (int)(ch & 1);
    if (ch + 1 < n_chunks) load_chunk(ch + 1);   // in flight during the MFMA work below
    const float* cb = cbuf + buf * TC * S;
#pragma unroll
    for (int t = 0; t < TC / 16; t += 2) {
      f32x4 acc[2][2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[tt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        float4 pv[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
          pv[tt] = *reinterpret_cast<const float4*>(cb + ((t + tt) * 16 + i) * S + c * 16 + 4 * g);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            acc[tt][nt] = mfma4(pv[tt].x, uf[nt][c].x, acc[tt][nt]);
            acc[tt][nt] = mfma4(pv[tt].y, uf[nt][c].y, acc[tt][nt]);
            acc[tt][nt] = mfma4(pv[tt].z, uf[nt][c].z, acc[tt][nt]);
            acc[tt][nt] = mfma4(pv[tt].w, uf[nt][c].w, acc[tt][nt]);
          }
      }
      // lane (i, g): acc[tt][nt][j] = score(candidate ch*TC + (t+tt)*16 + 4g + j, user nt*16 + i)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int64_t cbase = ch * TC + (t + tt) * 16 + 4 * g;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (cbase + j >= C) acc[tt][nt][j] = -__builtin_inff();   // never >= any thr
        bool any = false;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const f32x4 v = acc[tt][nt];
          any |= fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])) >= thr[nt];
        }
        if (__ballot(any) == 0ull) continue;   // wave-uniform: the common case
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float val = acc[tt][nt][j];
            unsigned long long cm = __ballot(val >= thr[nt]);
            while (cm) {
              const int src = __ffsll((long long)cm) - 1;
              const int u = nt * 16 + (src & 15);
              const float cs = __shfl(val, src, 64);
              const int ci = (int)(ch * TC + (t + tt) * 16 + 4 * (src >> 4) + j);
              float nthr;
              st_insert(lvw + u * L, liw + u * L, L, lane, cs, ci, nthr);
              if (i == (src & 15)) thr[nt] = fmaxf(thr[nt], nthr);
              cm = __ballot(val >= thr[nt]) & (~0ull << src << 1);
            }
          }
      }
    }
    if (ch + 1 < n_chunks) {
      // the other buffer held chunk ch - 1, which every wave finished before the barrier that
      // ended the previous iteration: one barrier per chunk
      store_chunk(buf ^ 1);
      __syncthreads();
    }
  }
  // write the lists
  for (int u = 0; u < kStUsersPerWave; ++u) {
    const int64_t r = row0 + u;
    if (r >= a.n_rows) break;
    if (lane < L) {
      a.topv[r * L + lane] = lvw[u * L + lane];
      a.topi[r * L + lane] = liw[u * L + lane];
    }
  }
}

// Metrics from the fused lists: one wave per row; rows where a tie crosses the cut get
// tie_flag = 1 and nothing else (the caller redoes them from materialised scores).
__global__ void __launch_bounds__(256) k_topk_finish(const TopkArgs a, const float* topv,
                                                     const int32_t* topi, int32_t L,
                                                     int32_t* tie_flag) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.n_rows) return;
  const int k = a.k;
  const float lvv = lane < L ? topv[row * L + lane] : -FLT_MAX;
  const int lii = lane < L ? topi[row * L + lane] : INT_MAX;
  const float tv = lane < k ? lvv : -FLT_MAX;
  const int ti = lane < k ? lii : INT_MAX;
  const float vnext = (a.n_cand > k) ? __shfl(lvv, k, 64) : -FLT_MAX;
  const bool done = row_metrics(a, row, lane, k, a.n_cand, tv, ti, vnext, nullptr);
  if (lane == 0) tie_flag[row] = done ? 0 : 1;
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_topk_metrics_rows(const float* scores, int64_t n_rows, int64_t n_cand, int64_t ld,
                           const int32_t* row_map, const int32_t* true_rowptr,
                           const int32_t* true_cand, const int32_t* true_count, int32_t K,
                           int32_t* topk_idx, double* recall, double* ndcg,
                           hgnn_stream_t stream_) {
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
  a.topk_idx = topk_idx; a.recall = recall; a.ndcg = ndcg; a.row_map = row_map;
  const dim3 grid((unsigned)cdiv(n_rows, 4)), block(256);
  hipLaunchKernelGGL(k_topk_metrics, grid, block, 0, stream, a);
  return check_launch("k_topk_metrics");
}

int hgnn_topk_metrics(const float* scores, int64_t n_rows, int64_t n_cand, int64_t ld,
                      const int32_t* true_rowptr, const int32_t* true_cand,
                      const int32_t* true_count, int32_t K, int32_t* topk_idx, double* recall,
                      double* ndcg, hgnn_stream_t stream) {
  return hgnn_topk_metrics_rows(scores, n_rows, n_cand, ld, nullptr, true_rowptr, true_cand,
                                true_count, K, topk_idx, recall, ndcg, stream);
}


size_t hgnn_score_topk_lds_bytes(int32_t d, int32_t L) {
  const int tc = 64, st = d + 8;
  return (size_t)2 * tc * st * 4 + (size_t)kStWaves * kStUsersPerWave * L * 8;
}

int hgnn_score_topk(const float* U, const int32_t* rows, int64_t n_rows, const float* P,
                    int64_t n_cand, int32_t d, int32_t L, float* topv, int32_t* topi,
                    hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_rows < 0 || n_cand < 1 || n_cand >= INT_MAX || L < 1 || L > 64 || L > n_cand)
    return fail(HGNN_E_ARG, "score_topk: rows=%lld cand=%lld L=%d", (long long)n_rows,
                (long long)n_cand, L);
  if (d != 64 && d != 128)
    return fail(HGNN_E_UNSUPPORTED, "score_topk: d=%d (64 or 128)", d);
  if (n_rows == 0) return HGNN_OK;
  if (!U || !P || !topv || !topi) return fail(HGNN_E_ARG, "score_topk: null pointer");
  if (reinterpret_cast<uintptr_t>(U) % 16 || reinterpret_cast<uintptr_t>(P) % 16)
    return fail(HGNN_E_ARG, "score_topk: U and P must be 16-B aligned");
  ScoreTopkArgs a{U, rows, n_rows, P, n_cand, L, topv, topi};
  const size_t lds = hgnn_score_topk_lds_bytes(d, L);
  const dim3 grid((unsigned)cdiv(n_rows, kStWaves * kStUsersPerWave)), block(kStThreads);
  if (d == 64) hipLaunchKernelGGL(k_score_topk<64>, grid, block, lds, stream, a);
  else hipLaunchKernelGGL(k_score_topk<128>, grid, block, lds, stream, a);
  return check_launch("k_score_topk");
}

int hgnn_topk_finish(const float* topv, const int32_t* topi, int64_t n_rows, int32_t L,
                     int64_t n_cand, int32_t K, const int32_t* true_rowptr,
                     const int32_t* true_cand, const int32_t* true_count, double* recall,
                     double* ndcg, int32_t* tie_flag, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  const int64_t k = K < n_cand ? K : n_cand;
  if (n_rows < 0 || K < 1 || K > 63 || n_cand < 1 || L != (n_cand > k ? k + 1 : k))
    return fail(HGNN_E_ARG, "topk_finish: rows=%lld K=%d L=%d cand=%lld (L must be "
                "min(K, cand) + 1, or min(K, cand) when cand <= K)", (long long)n_rows, K, L,
                (long long)n_cand);
  if (n_rows == 0) return HGNN_OK;
  if (!topv || !topi || !true_rowptr || !true_cand || !true_count || !recall || !ndcg ||
      !tie_flag)
    return fail(HGNN_E_ARG, "topk_finish: null pointer");
  TopkArgs a{};
  a.n_rows = n_rows; a.n_cand = n_cand; a.k = (int32_t)k;
  a.true_rowptr = true_rowptr; a.true_cand = true_cand; a.true_count = true_count;
  a.recall = recall; a.ndcg = ndcg;
  hipLaunchKernelGGL(k_topk_finish, dim3((unsigned)cdiv(n_rows, 4)), dim3(256), 0, stream, a,
                     topv, topi, L, tie_flag);
  return check_launch("k_topk_finish");
}

}  // extern "C"
