// Edge scoring + weighted BCE of the reference training step (train_gnn.py:259-281), fused.
//
//   s_pos[e] = <U[u_e], P[p_e]>,  s_neg[e] = <U[u_e], P[n_e]>
//   loss = mean(pos_weights) * mean_e softplus(-s_pos) + mean_e softplus(s_neg)
//
// (BCEWithLogitsLoss() reduces to a scalar, so the per-edge interaction weights collapse to their
// mean — the reference's own arithmetic, reproduced.)
//
// Pass A (this file) walks the positive edges grouped by user (the CSC of the engages relation):
// one wave per user keeps U[u] in registers, gathers P[p_e] and P[n_e] per edge, and in the same
// pass produces the loss partials AND dL/dU for a unit upstream gradient
//   dU[u] = sum_e  c/E (sigma(s_pos)-1) P[p_e] + 1/E sigma(s_neg) P[n_e]
// with no atomics (the wave owns the row).  It also emits each edge's weights for dP:
//   hpos (written at the edge's post-grouped position) and (n_e, u_e, hneg) for the negatives.
// dP is then two K1-style weighted gathers of U rows (gather.hip): positives over the post-
// grouped CSR, negatives over the (n_e)-sorted list (hgnn_sort_pairs_i32).  Deterministic.
#include "hgnn_common.h"

// Post rows of the negatives (uniform draws, little reuse) are read with nt loads: cfg4 scoring
// pass 26.4 -> 25.8 ms.  The positives' rows keep the default policy: their Zipf-hot posts live on
// cache reuse (nt on both: 33.1 ms).  Measurement builds: 0 = none, 2 = both.
// Cache policy (per launch, from the table sizes): the negatives' post rows (uniform draws,
// little reuse) are read with nt loads when the post table outgrows the Infinity Cache (cfg4,
// 488 MiB: 26.4 -> 25.8 ms; the positives' Zipf-hot rows keep the default policy: nt on both
// measured 33.1 ms); the dU rows are then stored nt too.  Its own instantiation, so the
// default-policy kernel (cfg2/cfg3) is the same code as before.


namespace hgnn {

struct ScoreArgs {
  const float* U;
  const float* P;
  const int32_t* rowptr;       // user-grouped CSR of the positive edges
  const int32_t* col;          // post id per position
  const int64_t* neg;          // negative post id per position (user-grouped order) ...
  const int32_t* neg32;        // ... or as int32 ...
  const uint64_t* neg_seed;    // ... or drawn here: uniform_draw(*neg_seed, position, n_posts)
  const int32_t* to_post_pos;  // position -> post-grouped position (for hpos)
  const float* cscale;         // device scalar mean(pos_weights)
  float* dU;
  float* hpos;
  int32_t* neg_key;
  int32_t* neg_u;
  float* neg_w;
  float* part;                 // [gridDim.x][2]
  int32_t* err;
  int64_t n_users;
  int64_t n_posts;
  float inv_e;
  int32_t d;
  int32_t nt_neg;              // nt policy: negatives' post rows loaded, dU rows stored
};

template <int LPR, int VPL, int W>
__device__ __forceinline__ float slot_dot(const typename Vec<W>::T (&a)[VPL],
                                          const typename Vec<W>::T (&b)[VPL]) {
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < VPL; ++q) {
    if constexpr (W == 4) {
      s = fmaf(a[q].x, b[q].x, s); s = fmaf(a[q].y, b[q].y, s);
      s = fmaf(a[q].z, b[q].z, s); s = fmaf(a[q].w, b[q].w, s);
    } else {
      s = fmaf(a[q], b[q], s);
    }
  }
  return slot_sum<LPR>(s);
}

template <int LPR, int VPL, int W, bool NT = false>
__global__ void __launch_bounds__(256) k_edge_score(const ScoreArgs a) {
  using V = Vec<W>;
  constexpr int NS = 64 / LPR;
  __shared__ float red[2][4];
  // wave index through readfirstlane: u, the row bounds and n are then scalar (wave-uniform to
  // the compiler), so the step loop's exits are scalar branches and the waitcnt pass can count
  // the in-flight prefetch across them
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int slot = lane / LPR, sl = lane % LPR;
  const int64_t u = (int64_t)blockIdx.x * 4 + wave;
  const float c = *a.cscale;
  const int d = a.d;
  // drawn negatives (hgnn_edge_score_fwd_draw): the draw of position k is recomputed here, so the
  // sort that groups them by post writes no position-order copy for this pass to read
  const bool seed_p = a.neg_seed != nullptr;
  const uint64_t seed = seed_p ? *a.neg_seed : 0;
  float lpos = 0.f, lneg = 0.f;   // per-lane loss sums (edge = lane)
  if (u < a.n_users) {
    const int64_t beg = a.rowptr[u], end = a.rowptr[u + 1];
    typename V::T uv[VPL], acc[VPL];
#pragma unroll
    for (int q = 0; q < VPL; ++q) {
      const int cc = (q * LPR + sl) * W;
      uv[q] = cc < d ? V::load(a.U + u * d + cc) : V::zero();
      acc[q] = V::zero();
    }
    for (int64_t base = beg; base < end; base += 64) {
      const int n = (int)min<int64_t>(64, end - base);
      int pid = 0, nid = 0;
      if (lane < n) {
        pid = a.col[base + lane];
        const int64_t nn = seed_p ? (int64_t)uniform_draw(seed, base + lane, (uint32_t)a.n_posts)
                           : a.neg32 ? (int64_t)a.neg32[base + lane] : a.neg[base + lane];
        if (nn < 0 || nn >= a.n_posts) {
          if (a.err) atomicAdd(a.err, 1);
        }
        else nid = (int)nn;
      }
      float my_hp = 0.f, my_hn = 0.f;
      // Software pipeline over steps of NS edges, two register sets in ping-pong: the rows of
      // step j+NS are in flight while step j is scored, with no register copy between steps (a
      // copy reads the prefetched registers, so it made each step wait for the next one's loads).
      // Loads are unconditional: lanes past the chunk read post 0 (pid/nid are 0 there) and
      // columns past d read column 0; neither reaches a result (their hp/hn are zeroed below, uv
      // is 0 past d, and the dU store is guarded).  Under exec-mask branches the compiler's
      // waitcnt pass could not count the prefetch and waited for it before using the previous
      // step's rows.
      typename V::T ap[VPL], an[VPL], bp[VPL], bn[VPL];
      auto load_step = [&](int j, typename V::T (&xp)[VPL], typename V::T (&xn)[VPL]) {
        const int e = j + slot;
        const int pp = __shfl(pid, e & 63, 64), qq = __shfl(nid, e & 63, 64);
#pragma unroll
        for (int q = 0; q < VPL; ++q) {
          const int cc = (q * LPR + sl) * W;
          const int ccl = cc < d ? cc : 0;
          xp[q] = V::load(a.P + (int64_t)pp * d + ccl);
          if constexpr (NT) xn[q] = V::load_nt(a.P + (int64_t)qq * d + ccl);
          else xn[q] = V::load(a.P + (int64_t)qq * d + ccl);
        }
      };
      auto score_step = [&](int j, const typename V::T (&vp)[VPL],
                            const typename V::T (&vn)[VPL]) {
        const int e = j + slot;
        const float sp = slot_dot<LPR, VPL, W>(uv, vp);
        const float sn = slot_dot<LPR, VPL, W>(uv, vn);
        const float tp = exp_neg_abs(sp), tn = exp_neg_abs(sn);
        float hp = c * a.inv_e * (sigmoid_t(sp, tp) - 1.f);
        float hn = a.inv_e * sigmoid_t(sn, tn);
        if (e >= n) hp = hn = 0.f;
        // loss terms once per edge, on the slot's first lane:
        //   softplus(-sp) = max(-sp, 0) + log(1 + t),  softplus(sn) = max(sn, 0) + log(1 + t)
        if (sl == 0 && e < n) {
          lpos += fmaxf(-sp, 0.f) + __logf(1.f + tp);
          lneg += fmaxf(sn, 0.f) + __logf(1.f + tn);
        }
#pragma unroll
        for (int q = 0; q < VPL; ++q) {
          V::fma(acc[q], hp, vp[q]);
          V::fma(acc[q], hn, vn[q]);
        }
        // hand edge e's weights to lane e (lanes j .. j+NS-1 read from slot lane*LPR)
        const int src = ((lane - j) & (NS - 1)) * LPR;
        const float thp = __shfl(hp, src, 64), thn = __shfl(hn, src, 64);
        if (lane >= j && lane < j + NS) {
          my_hp = thp; my_hn = thn;
        }
      };
      load_step(0, ap, an);
      for (int j = 0; j < n; j += 2 * NS) {
        load_step(j + NS, bp, bn);
        score_step(j, ap, an);
        if (j + NS >= n) break;
        load_step(j + 2 * NS, ap, an);
        score_step(j + NS, bp, bn);
      }
      if (lane < n) {
        const int64_t k = base + lane;
        if (a.hpos) a.hpos[a.to_post_pos[k]] = my_hp;
        if (a.neg_key) {
          a.neg_key[k] = nid;
          a.neg_u[k] = (int32_t)u;
        }
        if (a.neg_w) a.neg_w[k] = my_hn;
      }
    }
#pragma unroll
    for (int m = LPR; m < 64; m <<= 1)
#pragma unroll
      for (int q = 0; q < VPL; ++q) V::add(acc[q], V::shfl_xor(acc[q], m));
    if (lane < LPR) {
#pragma unroll
      for (int q = 0; q < VPL; ++q) {
        const int cc = (q * LPR + sl) * W;
        if (cc < d) {
          if constexpr (NT) V::store_nt(a.dU + u * d + cc, acc[q]);
          else V::store(a.dU + u * d + cc, acc[q]);
        }
      }
    }
  }
  // deterministic block partials: wave tree, then waves in order
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    lpos += __shfl_xor(lpos, m, 64);
    lneg += __shfl_xor(lneg, m, 64);
  }
  if (lane == 0) {
    red[0][wave] = lpos;
    red[1][wave] = lneg;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a.part[2 * blockIdx.x] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    a.part[2 * blockIdx.x + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
  }
}

// Deterministic two-level reduction of the block partials: 64 blocks each sum a contiguous
// range (double), then one block sums the 64 and forms the loss.
constexpr int kRedBlocks = 64;

__global__ void __launch_bounds__(256) k_loss_partial(const float* part, int64_t n_part,
                                                      double* red) {
  __shared__ double sp[256], sn[256];
  const int64_t per = cdiv(n_part, kRedBlocks);
  const int64_t b0 = blockIdx.x * per, b1 = min<int64_t>(b0 + per, n_part);
  double p = 0.0, q = 0.0;
  for (int64_t i = b0 + threadIdx.x; i < b1; i += 256) {
    p += part[2 * i];
    q += part[2 * i + 1];
  }
  sp[threadIdx.x] = p;
  sn[threadIdx.x] = q;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      sp[threadIdx.x] += sp[threadIdx.x + s];
      sn[threadIdx.x] += sn[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    red[2 * blockIdx.x] = sp[0];
    red[2 * blockIdx.x + 1] = sn[0];
  }
}

// loss = c * inv_e * sum(pos) + inv_e * sum(neg)
__global__ void k_loss_final(const double* red, const float* cscale, float inv_e, float* loss) {
  if (threadIdx.x != 0) return;
  double p = 0.0, q = 0.0;
  for (int i = 0; i < kRedBlocks; ++i) {
    p += red[2 * i];
    q += red[2 * i + 1];
  }
  *loss = (float)((double)*cscale * (double)inv_e * p + (double)inv_e * q);
}

// k_loss_partial + k_loss_final in one block (few partials: a sampled batch's loss), bitwise the
// same sums: wave w takes virtual blocks 4w .. 4w + 3; lane l stands for the partial kernel's
// threads l, l + 64, l + 128, l + 192 (the same strided double sums), the shared-memory tree's
// first two levels are in-lane adds and the other six shuffles in the same order; the 64 block
// sums are then added in order as k_loss_final does.
__global__ void __launch_bounds__(1024) k_loss_one(const float* part, int64_t n_part,
                                                   const float* cscale, float inv_e,
                                                   float* loss) {
  __shared__ double red[2 * kRedBlocks];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t per = cdiv(n_part, kRedBlocks);
  for (int vb = 4 * wv; vb < 4 * wv + 4; ++vb) {
    const int64_t b0 = vb * per, b1 = min<int64_t>(b0 + per, n_part);
    double p[4], q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      p[k] = 0.0;
      q[k] = 0.0;
      for (int64_t i = b0 + lane + 64 * k; i < b1; i += 256) {
        p[k] += part[2 * i];
        q[k] += part[2 * i + 1];
      }
    }
    // s = 128: t += t + 128 (slots 0, 1 take 2, 3); s = 64: slot 0 takes slot 1
    p[0] += p[2]; q[0] += q[2];
    p[1] += p[3]; q[1] += q[3];
    p[0] += p[1]; q[0] += q[1];
    double pp = p[0], qq = q[0];
    for (int s = 32; s > 0; s >>= 1) {   // t += t + s for t < s (lanes >= s carry don't-cares)
      const double po = __shfl_down(pp, s, 64), qo = __shfl_down(qq, s, 64);
      if (lane < s) {
        pp += po;
        qq += qo;
      }
    }
    if (lane == 0) {
      red[2 * vb] = pp;
      red[2 * vb + 1] = qq;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ps = 0.0, qs = 0.0;
    for (int i = 0; i < kRedBlocks; ++i) {
      ps += red[2 * i];
      qs += red[2 * i + 1];
    }
    *loss = (float)((double)*cscale * (double)inv_e * ps + (double)inv_e * qs);
  }
}

// few enough partials for one block to sum them faster than two launches
constexpr int64_t kLossOneMax = 65536;

template <int LPR, int VPL, int W>
static int launch_score(const ScoreArgs& a, int64_t nblocks, hipStream_t stream) {
  if (a.nt_neg)   // the cache policy as its own instantiation: the default one is unchanged
    hipLaunchKernelGGL((k_edge_score<LPR, VPL, W, true>), dim3((unsigned)nblocks), dim3(256), 0,
                       stream, a);
  else
    hipLaunchKernelGGL((k_edge_score<LPR, VPL, W>), dim3((unsigned)nblocks), dim3(256), 0,
                     stream, a);
  return check_launch("k_edge_score");
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

// floats of `part` scratch: 2 per block (4 users) + room for 2*64 doubles, 16-B aligned
int64_t hgnn_edge_score_parts(int64_t n_users) {
  return (int64_t)align_up((size_t)(2 * cdiv(n_users, 4)), 4) + 4 * kRedBlocks;
}

static int edge_score_fwd(const float* U, const float* P, int32_t d, int64_t n_users,
                          int64_t n_posts, const int32_t* rowptr_u, const int32_t* col_u,
                          const int64_t* neg_u_order, const int32_t* neg32,
                          const uint64_t* neg_seed, const int32_t* to_post_pos, int64_t n_edges, const float* cscale,
                          float* dU, float* hpos, int32_t* neg_key, int32_t* neg_user,
                          float* neg_w, float* part, float* loss, int32_t* err,
                          hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (d < 1 || n_users < 0 || n_posts < 0 || n_edges < 0)
    return fail(HGNN_E_ARG, "edge_score: bad sizes");
  if (!cscale || !loss ||
      (n_users > 0 && (!U || !rowptr_u || !dU || !part)) || (!neg_key != !neg_user))
    return fail(HGNN_E_ARG, "edge_score: null pointer");
  if (hpos && !to_post_pos) return fail(HGNN_E_ARG, "edge_score: hpos needs to_post_pos");
  if (err) (void)hipMemsetAsync(err, 0, sizeof(int32_t), stream);   // (null: not counted)
  ScoreArgs a{};
  a.U = U; a.P = P; a.rowptr = rowptr_u; a.col = col_u; a.neg = neg_u_order; a.neg32 = neg32;
  a.neg_seed = neg_seed;
  a.to_post_pos = to_post_pos; a.cscale = cscale; a.dU = dU; a.hpos = hpos; a.neg_key = neg_key;
  a.neg_u = neg_user; a.neg_w = neg_w; a.part = part; a.err = err; a.n_users = n_users;
  a.n_posts = n_posts; a.inv_e = n_edges > 0 ? 1.f / (float)n_edges : 0.f; a.d = d;
  a.nt_neg = n_posts * d * 4 >= (int64_t(256) << 20) ? 1 : 0;
  const int64_t nb = cdiv(n_users, 4);   // blocks of 4 user-waves
  int rc = HGNN_OK;
  if (nb > 0) {
    // one 4..16-edge step per iteration, next step's loads pipelined (an unrolled 2-step body
    // measured slower: users average ~20 edges, so wider steps waste the tail)
    if (d % 4 == 0 && d <= 64) rc = launch_score<16, 1, 4>(a, nb, stream);
    else if (d % 4 == 0 && d <= 128) rc = launch_score<32, 1, 4>(a, nb, stream);
    else if (d % 4 == 0 && d <= 256) rc = launch_score<64, 1, 4>(a, nb, stream);
    else if (d <= 64) rc = launch_score<64, 1, 1>(a, nb, stream);
    else if (d <= 512) rc = launch_score<64, 8, 1>(a, nb, stream);
    else return fail(HGNN_E_UNSUPPORTED, "edge_score: d=%d", d);
    if (rc) return rc;
  }
  // the reduction scratch lives after the block partials: part holds 2*nb floats + 2*64 doubles
  double* red = reinterpret_cast<double*>(part + align_up((size_t)(2 * nb), 4));
  if (nb <= kLossOneMax) {
    hipLaunchKernelGGL(k_loss_one, dim3(1), dim3(1024), 0, stream, part, nb, cscale, a.inv_e,
                       loss);
    return check_launch("k_loss_one");
  }
  hipLaunchKernelGGL(k_loss_partial, dim3(kRedBlocks), dim3(256), 0, stream, part, nb, red);
  if (int rc2 = check_launch("k_loss_partial")) return rc2;
  hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(64), 0, stream, red, cscale, a.inv_e, loss);
  return check_launch("k_loss_final");
}

int hgnn_edge_score_fwd(const float* U, const float* P, int32_t d, int64_t n_users,
                        int64_t n_posts, const int32_t* rowptr_u, const int32_t* col_u,
                        const int64_t* neg_u_order, const int32_t* to_post_pos, int64_t n_edges,
                        const float* cscale, float* dU, float* hpos, int32_t* neg_key,
                        int32_t* neg_user, float* neg_w, float* part, float* loss, int32_t* err,
                        hgnn_stream_t stream) {
  if (n_edges > 0 && !neg_u_order) return fail(HGNN_E_ARG, "edge_score: negatives are null");
  return edge_score_fwd(U, P, d, n_users, n_posts, rowptr_u, col_u, neg_u_order, nullptr,
                        nullptr, to_post_pos, n_edges, cscale, dU, hpos, neg_key, neg_user, neg_w, part,
                        loss, err, stream);
}

int hgnn_edge_score_fwd_i32(const float* U, const float* P, int32_t d, int64_t n_users,
                            int64_t n_posts, const int32_t* rowptr_u, const int32_t* col_u,
                            const int32_t* neg_u_order, int64_t n_edges, const float* cscale,
                            float* dU, float* part, float* loss, int32_t* err,
                            hgnn_stream_t stream) {
  if (n_edges > 0 && !neg_u_order) return fail(HGNN_E_ARG, "edge_score: negatives are null");
  return edge_score_fwd(U, P, d, n_users, n_posts, rowptr_u, col_u, nullptr, neg_u_order,
                        nullptr, nullptr, n_edges, cscale, dU, nullptr, nullptr, nullptr, nullptr, part,
                        loss, err, stream);
}

int hgnn_edge_score_fwd_draw(const float* U, const float* P, int32_t d, int64_t n_users,
                             int64_t n_posts, const int32_t* rowptr_u, const int32_t* col_u,
                             const uint64_t* d_seed, int64_t n_edges, const float* cscale,
                             float* dU, float* part, float* loss, int32_t* err,
                             hgnn_stream_t stream) {
  if (n_edges > 0 && !d_seed) return fail(HGNN_E_ARG, "edge_score: the draw's seed is null");
  if (n_posts < 1 || n_posts >= (int64_t(1) << 31) - 1)
    return fail(HGNN_E_ARG, "edge_score_draw: n_posts=%lld out of range", (long long)n_posts);
  return edge_score_fwd(U, P, d, n_users, n_posts, rowptr_u, col_u, nullptr, nullptr, d_seed,
                        nullptr, n_edges, cscale, dU, nullptr, nullptr, nullptr, nullptr, part,
                        loss, err, stream);
}

// Uniform draws in [0, hi): out[i] = hi * (splitmix64(seed + i * golden) >> 32) >> 32 (Lemire's
// multiply-shift), the seed read from device memory so the caller draws it from a torch
// Generator without a host sync.  The loss's negatives (train_gnn.py:272's torch.randint) drawn
// as int32 in range by construction: no int64 array, no validation pass before the sort.
__global__ void k_uniform_i32(const uint64_t* seed, int64_t n, uint32_t hi, int32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = uniform_draw(*seed, i, hi);
}

// x *= *s in place, skipped entirely when *s == 1 (read on the device: no host sync).  The
// loss's backward scales its precomputed dU/dP by the incoming gradient, which is exactly 1 for
// loss.backward(); the early exit turns a 256 MB read-modify-write into one launch.
__global__ void k_scale_unless_one(float* x, int64_t n, const float* s) {
  const float g = *s;
  if (g == 1.0f) return;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float4* x4 = reinterpret_cast<float4*>(x);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = x4[i];
    v.x *= g; v.y *= g; v.z *= g; v.w *= g;
    x4[i] = v;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    x[i] *= g;
}

int hgnn_scale_unless_one(float* x, int64_t n, const float* d_scale, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n < 0) return fail(HGNN_E_ARG, "scale_unless_one: n=%lld", (long long)n);
  if (n == 0) return HGNN_OK;
  if (!x || !d_scale) return fail(HGNN_E_ARG, "scale_unless_one: null pointer");
  if (reinterpret_cast<uintptr_t>(x) & 15)
    return fail(HGNN_E_ARG, "scale_unless_one: x must be 16-byte aligned");
  const int64_t blocks = std::min<int64_t>(cdiv(cdiv(n, 4), 256), 2048);
  hipLaunchKernelGGL(k_scale_unless_one, dim3((unsigned)blocks), dim3(256), 0, stream, x, n,
                     d_scale);
  return check_launch("k_scale_unless_one");
}

int hgnn_uniform_i32(const uint64_t* d_seed, int64_t n, int32_t hi, int32_t* out,
                     hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n < 0 || hi < 1) return fail(HGNN_E_ARG, "uniform_i32: n=%lld hi=%d", (long long)n, hi);
  if (n == 0) return HGNN_OK;
  if (!d_seed || !out) return fail(HGNN_E_ARG, "uniform_i32: null pointer");
  hipLaunchKernelGGL(k_uniform_i32, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, d_seed,
                     n, (uint32_t)hi, out);
  return check_launch("k_uniform_i32");
}

}  // extern "C"
