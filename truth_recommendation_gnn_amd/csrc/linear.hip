// K3/K4: fused multi-segment linear on fp32 MFMA (v_mfma_f32_16x16x4_f32, exact fp32 fma chain).
//
//   out[n, h] = act( sum_s X_s[n, K_s] @ W[:, off_s : off_s+K_s]^T + b )
//
// One call is a whole SAGE destination update: the segments are the per-relation mean
// aggregates and the destination's own features, W is the K-concatenation of the relation
// weights pre-scaled by the reference's fixed relation weights (train_gnn.py:163-164,187-198),
// act = ReLU.  That fuses lin_l + lin_r + weighted sum + bias + ReLU into one pass over HBM.
//
// MFMA operand trick: for a 16-wide K chunk, lane (i = lane&15, g = lane>>4) loads the float4
// X[row i][kc+4g .. kc+4g+3] and uses element q as the A operand of k-step q; B takes the same
// k from W.  So k-step q sums k = kc+4g+q over g — every k of the chunk exactly once, with
// contiguous 16-B loads (the k order inside a chunk is permuted, which only moves rounding).
#include "linear_common.h"

#include <algorithm>
#include <stdlib.h>

namespace hgnn {


__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}


template <bool VEC>
__device__ __forceinline__ void load4(const float* p, int valid_elems, float (&v)[4]) {
  if (VEC) {
    if (valid_elems >= 4) {
      float4 t = *reinterpret_cast<const float4*>(p);
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
      v[0] = v[1] = v[2] = v[3] = 0.f;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = q < valid_elems ? p[q] : 0.f;
  }
}

constexpr int RT = 2;             // 16-row tiles per wave
constexpr int kRowsPerBlock = 4 * RT * 16;

// ---------------------------------------------------------------- forward
template <int NT, bool VEC>
__global__ void __launch_bounds__(256) k_linear_fwd(const LinArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock + wave * (RT * 16);
  const int c0 = blockIdx.y * (NT * 16);
  f32x4 acc[RT][NT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < a.n_seg; ++s) {
    const Seg sg = a.seg[s];
    for (int kc = 0; kc < sg.k; kc += 16) {
      const int k = kc + 4 * g;
      const int kv = sg.k - k;  // valid elements from k
      float av[RT][4], bv[NT][4];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int64_t row = r0 + rt * 16 + i;
        if (row < a.n) load4<VEC>(sg.x + row * sg.k + k, kv, av[rt]);
        else av[rt][0] = av[rt][1] = av[rt][2] = av[rt][3] = 0.f;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int col = c0 + t * 16 + i;
        if (col < a.h) load4<VEC>(a.w + (int64_t)col * a.k_total + sg.off + k, kv, bv[t]);
        else bv[t][0] = bv[t][1] = bv[t][2] = bv[t][3] = 0.f;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[rt][t] = mfma4(av[rt][q], bv[t][q], acc[rt][t]);
    }
  }
  // C/D map of 16x16x4: col = lane&15, row = 4*(lane>>4) + reg
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = c0 + t * 16 + i;
    if (col >= a.h) continue;
    const float b = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t row = r0 + rt * 16 + 4 * g + j;
        if (row < a.n) {
          float v = acc[rt][t][j] + b;
          if (a.relu) v = fmaxf(v, 0.f);
          a.out[row * a.h + col] = v;
        }
      }
  }
}

// Forward variant: W staged once per 128-row block in LDS, each wave's A fragments for the whole
// K (<= 128, every segment a multiple of 16) loaded up front, so the MFMA loop never waits on
// global memory; B fragments by ds_read_b128.
template <int NT, int KC>
__global__ void __launch_bounds__(256) k_linear_fwd_v2(const LinArgs a) {
  extern __shared__ __attribute__((aligned(16))) float ws[];   // [h][K+4]
  const int K = a.k_total, ldw = K + 4;
  for (int idx = threadIdx.x; idx < a.h * (K >> 2); idx += 256) {
    const int j = idx / (K >> 2), k = (idx - j * (K >> 2)) * 4;
    *reinterpret_cast<float4*>(ws + j * ldw + k) =
        *reinterpret_cast<const float4*>(a.w + (int64_t)j * K + k);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock + wave * (RT * 16);
  float4 av[RT][KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int k = c * 16;
    int s = 0;
    while (s + 1 < a.n_seg && k >= a.seg[s].off + a.seg[s].k) ++s;
    const float* xs = a.seg[s].x;
    const int ks = a.seg[s].k, kk = k - a.seg[s].off + 4 * g;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int64_t row = r0 + rt * 16 + i;
      av[rt][c] = row < a.n ? *reinterpret_cast<const float4*>(xs + row * ks + kk)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();
  f32x4 acc[RT][NT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < KC; ++c) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float4 bv = *reinterpret_cast<const float4*>(ws + (t * 16 + i) * ldw + c * 16 + 4 * g);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        acc[rt][t] = mfma4(av[rt][c].x, bv.x, acc[rt][t]);
        acc[rt][t] = mfma4(av[rt][c].y, bv.y, acc[rt][t]);
        acc[rt][t] = mfma4(av[rt][c].z, bv.z, acc[rt][t]);
        acc[rt][t] = mfma4(av[rt][c].w, bv.w, acc[rt][t]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = t * 16 + i;
    const float b = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t row = r0 + rt * 16 + 4 * g + j;
        if (row < a.n) {
          float v = acc[rt][t][j] + b;
          if (a.relu) v = fmaxf(v, 0.f);
          a.out[row * a.h + col] = v;
        }
      }
  }
}

// ---------------------------------------------------------------- dgrad: dX_s = dZ @ W_s
template <bool VEC>
__device__ __forceinline__ void load_dz(const LinArgs& a, int64_t row, int j, float (&v)[4]) {
  const int jv = a.h - j;
  if (row >= a.n) { v[0] = v[1] = v[2] = v[3] = 0.f; return; }
  load4<VEC>(a.dout + row * a.h + j, jv, v);
  if (a.out_act) {
    float m[4];
    load4<VEC>(a.out_act + row * a.h + j, jv, m);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = m[q] > 0.f ? v[q] : 0.f;
  }
}

template <int NT, bool VEC>
__global__ void __launch_bounds__(256) k_linear_dgrad(const LinArgs a) {
  const int c0 = blockIdx.y * (NT * 16);
  bool any = false;
  for (int s = 0; s < a.n_seg; ++s)
    any |= a.seg[s].dx && a.seg[s].off < c0 + NT * 16 && a.seg[s].off + a.seg[s].k > c0;
  if (!any) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock + wave * (RT * 16);
  f32x4 acc[RT][NT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int jc = 0; jc < a.h; jc += 16) {
    const int j = jc + 4 * g;
    float av[RT][4], bv[NT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) load_dz<VEC>(a, r0 + rt * 16 + i, j, av[rt]);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = c0 + t * 16 + i;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        bv[t][q] = (col < a.k_total && j + q < a.h) ? a.w[(int64_t)(j + q) * a.k_total + col]
                                                    : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[rt][t] = mfma4(av[rt][q], bv[t][q], acc[rt][t]);
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = c0 + t * 16 + i;
    if (col >= a.k_total) continue;
    int s = 0;
    while (s + 1 < a.n_seg && col >= a.seg[s].off + a.seg[s].k) ++s;
    float* dx = a.seg[s].dx;
    if (!dx) continue;
    const int kk = col - a.seg[s].off, ks = a.seg[s].k;
    const bool add = (a.dx_acc >> s) & 1u;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int64_t row = r0 + rt * 16 + 4 * g + jj;
        if (row < a.n) {
          float* p = dx + row * ks + kk;
          *p = add ? *p + acc[rt][t][jj] : acc[rt][t][jj];
        }
      }
  }
}

// ---------------------------------------------------------------- wgrad partials
// Block: 4 waves, j range of 64 (blockIdx.z), k range of 128 over [X_0..X_{S-1}, 1] (blockIdx.y;
// the trailing ones column gives db), rows [bx*rows_per_block, ...) staged 32 at a time in LDS.
constexpr int WG_ROWS = 32;
constexpr int WG_J = 64;
constexpr int WG_K = 128;
constexpr int DZ_LD = WG_J + 16;   // row stride = 16 mod 32 banks: lanes g and g+1 disjoint
constexpr int X_LD = WG_K + 16;

template <bool VEC>
__global__ void __launch_bounds__(256) k_linear_wgrad(const LinArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[WG_ROWS * DZ_LD + WG_ROWS * X_LD];
  float* dz_l = lds;
  float* x_l = lds + WG_ROWS * DZ_LD;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int j0 = blockIdx.z * WG_J, k0 = blockIdx.y * WG_K;
  const int kext = a.k_total + 1;
  const int64_t rb = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t re = min<int64_t>(rb + a.rows_per_block, a.n);
  f32x4 acc[WG_K / 16];
#pragma unroll
  for (int t = 0; t < WG_K / 16; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t rs = rb; rs < re; rs += WG_ROWS) {
    // stage dZ[32][64] (masked) and X[32][128]: one float4 per (row, 4 columns)
    for (int idx = threadIdx.x; idx < WG_ROWS * (WG_J / 4); idx += 256) {
      const int r = idx / (WG_J / 4), c4 = idx % (WG_J / 4);
      float v[4];
      load_dz<VEC>(a, rs + r < re ? rs + r : a.n, j0 + 4 * c4, v);
      *reinterpret_cast<float4*>(dz_l + r * DZ_LD + 4 * c4) = make_float4(v[0], v[1], v[2], v[3]);
    }
    for (int idx = threadIdx.x; idx < WG_ROWS * (WG_K / 4); idx += 256) {
      const int r = idx / (WG_K / 4), c4 = idx % (WG_K / 4);
      const int64_t row = rs + r;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (row < re) {
        const int kg = k0 + 4 * c4;
        if (VEC && kg + 4 <= a.k_total) {
          int s = 0;
          while (s + 1 < a.n_seg && kg >= a.seg[s].off + a.seg[s].k) ++s;
          const float4 t =
              *reinterpret_cast<const float4*>(a.seg[s].x + row * a.seg[s].k + kg - a.seg[s].off);
          v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int kq = kg + q;
            if (kq < a.k_total) {
              int s = 0;
              while (s + 1 < a.n_seg && kq >= a.seg[s].off + a.seg[s].k) ++s;
              v[q] = a.seg[s].x[row * a.seg[s].k + kq - a.seg[s].off];
            } else if (kq == a.k_total) {
              v[q] = 1.f;
            }
          }
        }
      }
      *reinterpret_cast<float4*>(x_l + r * X_LD + 4 * c4) = make_float4(v[0], v[1], v[2], v[3]);
    }
    __syncthreads();
    // A[i = j][kk = row] = dZ[row][j], B[kk = row][col = k] = X[row][k]; k-step s covers rows 4s..4s+3
#pragma unroll
    for (int s = 0; s < WG_ROWS / 4; ++s) {
      const int r = 4 * s + g;
      const float av = dz_l[r * DZ_LD + wave * 16 + i];
#pragma unroll
      for (int t = 0; t < WG_K / 16; ++t) acc[t] = mfma4(av, x_l[r * X_LD + t * 16 + i], acc[t]);
    }
    __syncthreads();
  }
  // partial tile: rows j = j0 + wave*16 + 4g + jj, cols k = k0 + 16t + i
  float* slab = a.slab + (int64_t)blockIdx.x * a.h * kext;
#pragma unroll
  for (int t = 0; t < WG_K / 16; ++t) {
    const int k = k0 + t * 16 + i;
    if (k >= kext) continue;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = j0 + wave * 16 + 4 * g + jj;
      if (j < a.h) slab[(int64_t)j * kext + k] = acc[t][jj];
    }
  }
}

// dw[j][k] = sum_b slab[b][j][k] (k < K), db[j] = sum_b slab[b][j][K]; fixed b order.
// ldd: dw's row stride (kext - 1, or the whole dW's K for a column block of it)
__device__ __forceinline__ void wgrad_reduce_body(const float* slab, int64_t nb, int32_t h,
                                                  int32_t kext, float* dw, float* db, int32_t ldd,
                                                  int64_t bid) {
  // 64 outputs per block (lanes), 16 waves each sum a contiguous range of slabs with 4
  // independent accumulators, then wave 0 adds the 16 partials in order: a fixed summation
  // order for a given nb (deterministic), and enough loads in flight to stream the slabs
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t e = bid * 64 + lane;
  const int64_t total = (int64_t)h * kext;
  const int64_t per = cdiv(nb, 16);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (e < total) {
    const int64_t b1 = min<int64_t>((wave + 1) * per, nb);
    int64_t b = wave * per;
    for (; b + 4 <= b1; b += 4) {
      s0 += slab[b * total + e];
      s1 += slab[(b + 1) * total + e];
      s2 += slab[(b + 2) * total + e];
      s3 += slab[(b + 3) * total + e];
    }
    for (; b < b1; ++b) s0 += slab[b * total + e];
  }
  part[wave][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (wave == 0 && e < total) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) v += part[w][lane];
    const int j = (int)(e / kext), k = (int)(e % kext);
    if (k < kext - 1) { if (dw) dw[(int64_t)j * ldd + k] = v; }
    else if (db) db[j] = v;
  }
}

__global__ void __launch_bounds__(1024) k_wgrad_reduce(const float* slab, int64_t nb, int32_t h,
                                                       int32_t kext, float* dw, float* db,
                                                       int32_t ldd) {
  wgrad_reduce_body(slab, nb, h, kext, dw, db, ldd, blockIdx.x);
}

// Two jobs' slabs (the split kernels' two-job backward) in one launch: blocks [0, nblk0) reduce
// job 0, the rest job 1 — each output the same sum in the same order as a launch of its own.
struct ReducePair {
  const float* slab[2];
  int64_t nb[2];
  float* dw[2];
  float* db[2];
  int64_t nblk0;
  int32_t h, kext, ldd;
};
__global__ void __launch_bounds__(1024) k_wgrad_reduce2(const ReducePair p) {
  if ((int64_t)blockIdx.x < p.nblk0)
    wgrad_reduce_body(p.slab[0], p.nb[0], p.h, p.kext, p.dw[0], p.db[0], p.ldd, blockIdx.x);
  else
    wgrad_reduce_body(p.slab[1], p.nb[1], p.h, p.kext, p.dw[1], p.db[1], p.ldd,
                      (int64_t)blockIdx.x - p.nblk0);
}

// ================================================================ fused backward (LDS path)
// When W fits in LDS (h*K*4 <= 64 KiB), h % 16 == 0, K % 32 == 0 and every segment is float4-
// aligned: persistent blocks keep W^T resident in LDS and stream 32-row tiles of dz and X
// through LDS once (register prefetch of the next tile overlaps HBM with the MFMAs), computing
// dX and the block's dW/db from the same staged tiles.  (An LDS-staged forward built the same
// way measured no faster than the direct-fragment forward — 345 vs 325 us at N=1M, K=128, h=64,
// both MFMA-issue bound at ~50 TF/s — so the forward keeps the direct kernel.)
constexpr int FT = 32;  // rows per tile

// Register prefetch of one [FT x K] tile (K <= 128 => at most 4 float4 per thread): issued
// before the current tile's MFMAs so HBM latency overlaps compute, stored to LDS after.
struct XPrefetch {
  float4 v[4];
  __device__ __forceinline__ void load(const LinArgs& a, int64_t r0) {
    const int k4 = a.k_total >> 2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = threadIdx.x + 256 * q;
      v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (idx < FT * k4) {
        const int r = idx / k4, k = (idx - r * k4) * 4;
        int s = 0;
        while (s + 1 < a.n_seg && k >= a.seg[s].off + a.seg[s].k) ++s;
        const int64_t row = r0 + r;
        if (row < a.n)
          v[q] = *reinterpret_cast<const float4*>(a.seg[s].x + row * a.seg[s].k +
                                                  (k - a.seg[s].off));
      }
    }
  }
  __device__ __forceinline__ void store(const LinArgs& a, float* xs, int ld) const {
    const int k4 = a.k_total >> 2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = threadIdx.x + 256 * q;
      if (idx < FT * k4) {
        const int r = idx / k4, k = (idx - r * k4) * 4;
        *reinterpret_cast<float4*>(xs + r * ld + k) = v[q];
      }
    }
  }
};

// Fused backward: per 32-row tile, dz = dout * (out > 0) and X staged once; dX = dz @ W (W^T in
// LDS) and the block's dW (+ db as the column K) accumulated in registers across its tiles,
// written once as a partial [h][K+1] slab (reduced in block order by k_wgrad_reduce).
template <int NT, bool DX>
__global__ void __launch_bounds__(256) k_linear_bwd_lds(const LinArgs a, int64_t n_tiles) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = a.k_total, h = a.h;
  const int ldwt = h + 4, ldz = h + 16, ldx = K + 16;   // b32 reads: row stride = 16 mod 32
  float* wt = smem;                 // [K][ldwt]  W^T
  float* dz = wt + K * ldwt;        // [FT][ldz]
  float* xs = dz + FT * ldz;        // [FT][ldx]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  constexpr int JT = NT >= 4 ? NT / 4 : 1;      // j tiles per wave (wgrad)
  const bool wave_has_j = NT >= 4 || wave < NT;
  const int KT = K >> 4;
  if (DX) {
    for (int idx = threadIdx.x; idx < h * K; idx += 256) {
      const int j = idx / K, k = idx - j * K;
      wt[k * ldwt + j] = a.w[(int64_t)j * K + k];
    }
  }
  f32x4 acc[JT][8];   // K <= 128 on this path
#pragma unroll
  for (int jt = 0; jt < JT; ++jt)
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) acc[jt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 dbacc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int h4 = h >> 2;
  // prefetch registers: dz (dout masked by out) <= 4 float4, X <= 4 float4 per thread
  float4 zp[4];
  XPrefetch pf;
  auto load_dz = [&](int64_t r0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = threadIdx.x + 256 * q;
      zp[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (idx < FT * h4) {
        const int r = idx / h4, c = (idx - r * h4) * 4;
        const int64_t row = r0 + r;
        if (row < a.n) {
          float4 v = *reinterpret_cast<const float4*>(a.dout + row * h + c);
          if (a.out_act) {
            const float4 m = *reinterpret_cast<const float4*>(a.out_act + row * h + c);
            v.x = m.x > 0.f ? v.x : 0.f; v.y = m.y > 0.f ? v.y : 0.f;
            v.z = m.z > 0.f ? v.z : 0.f; v.w = m.w > 0.f ? v.w : 0.f;
          }
          zp[q] = v;
        }
      }
    }
  };
  load_dz((int64_t)blockIdx.x * FT);
  pf.load(a, (int64_t)blockIdx.x * FT);
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t r0 = tile * FT;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = threadIdx.x + 256 * q;
      if (idx < FT * h4) {
        const int r = idx / h4, c = (idx - r * h4) * 4;
        const float4 v = zp[q];
        dbacc.x += v.x; dbacc.y += v.y; dbacc.z += v.z; dbacc.w += v.w;
        *reinterpret_cast<float4*>(dz + r * ldz + c) = v;
      }
    }
    pf.store(a, xs, ldx);
    __syncthreads();
    if (tile + gridDim.x < n_tiles) {
      load_dz((tile + gridDim.x) * FT);
      pf.load(a, (tile + gridDim.x) * FT);
    }
    if (DX) {   // dX tile [FT x K]: wave = row tile (wave & 1) x column half (wave >> 1)
      const int rt = wave & 1, half = wave >> 1;
      const int ct0 = half * (KT >> 1), nct = KT >> 1;
      for (int c = 0; c < nct; ++c) {
        const int ct = ct0 + c;
        f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int jc = 0; jc < h; jc += 16) {
          const float4 av = *reinterpret_cast<const float4*>(dz + (rt * 16 + i) * ldz + jc + 4 * g);
          const float4 bv = *reinterpret_cast<const float4*>(wt + (ct * 16 + i) * ldwt + jc + 4 * g);
          o = mfma4(av.x, bv.x, o);
          o = mfma4(av.y, bv.y, o);
          o = mfma4(av.z, bv.z, o);
          o = mfma4(av.w, bv.w, o);
        }
        const int col = ct * 16 + i;
        int s = 0;
        while (s + 1 < a.n_seg && col >= a.seg[s].off + a.seg[s].k) ++s;
        float* dx = a.seg[s].dx;
        if (dx) {
          const int kk = col - a.seg[s].off, ks = a.seg[s].k;
          const bool add = (a.dx_acc >> s) & 1u;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int64_t row = r0 + rt * 16 + 4 * g + r;
            if (row < a.n) {
              float* p = dx + row * ks + kk;
              *p = add ? *p + o[r] : o[r];
            }
          }
        }
      }
    }
    if (wave_has_j) {   // wgrad: A[i=j][kk=row] = dz[row][j], B[kk=row][col=k] = X[row][k]
#pragma unroll 2
      for (int s4 = 0; s4 < FT / 4; ++s4) {
        const int r = 4 * s4 + g;
        float bv[8];
#pragma unroll
        for (int kt = 0; kt < 8; ++kt) bv[kt] = kt < KT ? xs[r * ldx + kt * 16 + i] : 0.f;
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
          const float av = dz[r * ldz + (wave + 4 * jt) * 16 + i];
#pragma unroll
          for (int kt = 0; kt < 8; ++kt)
            if (kt < KT) acc[jt][kt] = mfma4(av, bv[kt], acc[jt][kt]);
        }
      }
    }
  }
  // partial slab [blockIdx.x][h][K+1]
  const int kext = K + 1;
  float* slab = a.slab + (int64_t)blockIdx.x * h * kext;
  if (wave_has_j) {
#pragma unroll
    for (int jt = 0; jt < JT; ++jt)
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) {
        if (kt >= KT) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = (wave + 4 * jt) * 16 + 4 * g + r;
          slab[(int64_t)j * kext + kt * 16 + i] = acc[jt][kt][r];
        }
      }
  }
  __syncthreads();
  float4* red = reinterpret_cast<float4*>(xs);     // [256] thread partials of db
  red[threadIdx.x] = dbacc;
  __syncthreads();
  if (threadIdx.x < h4) {   // thread t staged columns 4*(t % h4) on every tile
    float4 t = red[threadIdx.x];
    for (int m = threadIdx.x + h4; m < 256; m += h4) {
      const float4 u = red[m];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    const int c = threadIdx.x * 4;
    slab[(int64_t)(c + 0) * kext + K] = t.x;
    slab[(int64_t)(c + 1) * kext + K] = t.y;
    slab[(int64_t)(c + 2) * kext + K] = t.z;
    slab[(int64_t)(c + 3) * kext + K] = t.w;
  }
}

// The bf16x6 K3 kernels (H = 128, K = 128 / 256): on unless HGNN_K3_X6=0, or as last set by
// hgnn_set_k3_split (tests run both paths in one process).
static int g_k3_x6 = -1;
static bool x6_enabled() {
  if (g_k3_x6 < 0) g_k3_x6 = (!getenv("HGNN_K3_X6") || atoi(getenv("HGNN_K3_X6")) != 0) ? 1 : 0;
  return g_k3_x6 != 0;
}

static bool fast_path_ok(const LinArgs& a, bool vec) {
  static const int off = getenv("HGNN_LIN_GENERAL") ? atoi(getenv("HGNN_LIN_GENERAL")) : 0;
  if (off) return false;
  return vec && a.h % 16 == 0 && a.h <= 128 && a.k_total % 32 == 0 && a.k_total <= 128 &&
         (size_t)a.h * a.k_total * 4 <= 65536 && 256 % (a.h / 4) == 0;
}

static int fast_grid(int64_t n_tiles) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(n_tiles, 512));
}

// ================================================================ v4: compile-time shapes
// H (output width) in {64, 128}, K (sum of segments) in {64, 128, 256}, every segment a multiple
// of 16 columns and float4-aligned.  Per 16-column chunk c of the concatenated input, a host-built
// table gives the segment base/stride (no per-element segment search).
// LDS strides are chosen so that addresses stay affine in the lane id (the compiler keeps one
// base register + immediates) and the two access kinds are conflict-free:
//   * ds_read_b128 where lanes (i, g) read row i, columns 4g..4g+3: stride = 8 (mod 16) dwords
//     (row i lands on 16-B slot 2i + g: even/odd by g, 8 distinct per b128 lane group);
//   * ds_read_b32 where lanes (i, g) read row g, column i: stride = 16 (mod 32) dwords.


// Address of row `row`'s float4 at columns 16 c + 4 g .. +3 of the concatenated input.  S8: every
// 8 consecutive chunks are one segment (segments 128 columns wide, as at cfg3/cfg4), so with c
// unrolled the row offset is one multiply per segment and the chunks are immediates off it
// (the general form keeps a 64-bit address per chunk live across the MFMA sweep).
template <bool S8>
__device__ __forceinline__ const float4* x_chunk(const ChunkTab& tab, int64_t row, int c, int g) {
  if constexpr (S8) {
    const int s = c & ~7;
    return reinterpret_cast<const float4*>(tab.x[s] + row * tab.ld[s] + tab.col[s] +
                                           (c & 7) * 16 + 4 * g);
  } else {
    return reinterpret_cast<const float4*>(tab.x[c] + row * tab.ld[c] + tab.col[c] + 4 * g);
  }
}

// The added rows of one 16-row tile (hgnn_linear_fwd_add: a pre-projected relation's gathered
// mean), loaded before the tile's MFMA sweep, which hides their HBM latency; read in the
// epilogue they stalled every tile (K = 128 + add ran at 0.53 of the fp32 MFMA peak).  Lane
// (i, g) holds columns 16 tt + 4 g .. +3 of its row.  The bias stays an epilogue read (L1-hot).
template <int NT, bool ADD>
struct Epi {
  float4 d[ADD ? NT : 1];
  __device__ __forceinline__ void load(const LinArgs& a, int64_t row, int H, int g) {
    if constexpr (ADD) {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
        d[tt] = row < a.n ? *reinterpret_cast<const float4*>(a.add + row * H + tt * 16 + 4 * g)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // (acc + bias) + add: the order of the unfused expression
  __device__ __forceinline__ float4 sum(const f32x4& acc, int tt, const LinArgs& a, int g) const {
    const float4 bb = a.bias ? *reinterpret_cast<const float4*>(a.bias + tt * 16 + 4 * g)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v = make_float4(acc[0] + bb.x, acc[1] + bb.y, acc[2] + bb.z, acc[3] + bb.w);
    if constexpr (ADD) {
      v.x += d[tt].x; v.y += d[tt].y; v.z += d[tt].z; v.w += d[tt].w;
    }
    return v;
  }
};

// Forward v4: persistent.  W is staged into LDS once per block; then each of the 8 waves streams
// its own 16-row tiles (no further barriers), with the next tile's A fragments in flight during
// the current tile's MFMAs.  (Measured and rejected: MFMAs interleaved across accumulators —
// the 4-deep dependent chains are already covered by 4 waves per SIMD — and a two-stage register
// ping-pong instead of the copy, which spills: 193-200 us vs 202-205 and 227 at N=1M, K=128.)  Output tiles are computed transposed (out^T = W X^T) so every lane
// stores one float4 per 16 output columns.
template <int H, int K, bool ADD, bool S8 = false>
__global__ void __launch_bounds__(512, (H <= 64 && K <= 128 ? 4 : (K <= 128 ? 3 : 2))) k_linear_fwd_v4(const LinArgs a, const ChunkTab tab,
                                                       int64_t n_tiles) {
  constexpr int NT = H / 16, KC = K / 16, LDW = K + 8;
  __shared__ __attribute__((aligned(16))) float ws[H * LDW];
  for (int idx = threadIdx.x; idx < H * K / 4; idx += 512) {
    const int j = idx / (K / 4), k = (idx % (K / 4)) * 4;
    *reinterpret_cast<float4*>(ws + j * LDW + k) =
        *reinterpret_cast<const float4*>(a.w + (int64_t)j * K + k);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int64_t nw = (int64_t)gridDim.x * 8;
  auto load = [&](int64_t t, float4 (&v)[KC]) {
    const int64_t row = t * 16 + i;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      v[c] = row < a.n ? *x_chunk<S8>(tab, row, c, g) : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  int64_t t = (int64_t)blockIdx.x * 8 + wave;
  float4 av[KC], an[KC];
  if (t < n_tiles) load(t, av);
  __syncthreads();
  const int wl0 = i * LDW + 4 * g;
  for (; t < n_tiles; t += nw) {
    if (t + nw < n_tiles) load(t + nw, an);
    // opaque offset: keeps the loop-invariant W fragments as per-tile LDS reads instead of letting
    // the compiler hoist all K*H/64 of them into VGPRs (measured 195 vs 204 us at N=1M, K=128, H=64,
    // and no spill at H=128)
    int wo = wl0;
    asm volatile("" : "+v"(wo));
    const float* wl = ws + wo;
    const int64_t row = t * 16 + i;
    Epi<NT, ADD> ep;               // the added rows, in flight during the sweep
    ep.load(a, row, H, g);
    f32x4 acc[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < KC; ++c)
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        const float4 bv = *reinterpret_cast<const float4*>(wl + tt * 16 * LDW + c * 16);
        acc[tt] = mfma4(bv.x, av[c].x, acc[tt]);
        acc[tt] = mfma4(bv.y, av[c].y, acc[tt]);
        acc[tt] = mfma4(bv.z, av[c].z, acc[tt]);
        acc[tt] = mfma4(bv.w, av[c].w, acc[tt]);
      }
    if (row < a.n) {
      uint32_t mbits = 0;   // ReLU mask bits of this lane's columns (mask_out)
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        float4 v = ep.sum(acc[tt], tt, a, g);
        if (a.relu) {
          v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        }
        mbits |= relu_bits(v, 4 * tt);
        *reinterpret_cast<float4*>(a.out + row * H + tt * 16 + 4 * g) = v;
      }
      if (a.mask_out) a.mask_out[row * 4 + g] = mbits;
    }
#pragma unroll
    for (int c = 0; c < KC; ++c) av[c] = an[c];
  }
}

// Backward v4: two roles per SIMD.  512 threads; waves 0-3 ("dz waves") load the masked dz
// fragments of 16 rows each, run dgrad (dX^T = W^T dz^T, straight from registers) and the bias
// sums, and publish dz to LDS; waves 4-7 ("X waves") stage the X tile and run wgrad.  dz / X
// tiles are double-buffered, so with one barrier per tile the dgrad of tile t+1 (dz waves) runs
// beside the wgrad of tile t (X waves) on every SIMD: MFMA issue from one role hides the memory
// waits of the other.
// T = 32 (wgrad-only, for K = 256 whose X tiles would not fit twice at T = 64): the two 16-row
// slices of a tile go to dz waves (w & 1), each loading half of the columns (w >> 1).
template <int H, int K, bool DX, int T = 64>
__global__ void __launch_bounds__(512) k_linear_bwd_v4(const LinArgs a, const ChunkTab tab,
                                                       int64_t n_tiles) {
  static_assert(T == 64 || (T == 32 && !DX), "dgrad needs one 16-row slice per dz wave");
  constexpr int HC = H / 16, KC = K / 16;
  constexpr int ZR = T / 16;                // 16-row slices per tile
  constexpr int ZC = HC * ZR / 4;           // column chunks loaded per dz wave
  constexpr int JT = H / 64;                // wgrad j tiles per X wave
  constexpr int XQ = T * K / 4 / 256;       // X float4 per X-wave thread per tile
  constexpr int LWT = H + 8, LZ = H + 16, LX = K + 16;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* wt = smem;                         // [K][LWT]  W^T   (DX only)
  float* dzb = wt + (DX ? K * LWT : 0);     // 2 x [T][LZ]
  float* xsb = dzb + 2 * T * LZ;            // 2 x [T][LX]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const bool zrole = wave < 4;
  const int w4 = wave & 3;
  const int zrow = w4 % ZR, zcol0 = (w4 / ZR) * ZC;   // dz wave: row slice, first column chunk
  if (DX) {
    for (int idx = threadIdx.x; idx < H * K; idx += 512) {
      const int j = idx / K, k = idx % K;
      wt[k * LWT + j] = a.w[(int64_t)j * K + k];
    }
    __syncthreads();   // block-uniform: W^T image complete before the first dgrad
  }
  const int64_t n_my = (n_tiles - blockIdx.x + gridDim.x - 1) / gridDim.x;
  if (zrole) {
    auto load_dz = [&](int64_t it, float4 (&z)[HC]) {
      const int64_t row = (blockIdx.x + it * gridDim.x) * T + zrow * 16 + i;
      const uint32_t mk = a.mask_in && it < n_my && row < a.n ? a.mask_in[row * 4 + g] : 0u;
#pragma unroll
      for (int c = 0; c < HC; ++c) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (it < n_my && row < a.n && c >= zcol0 && c < zcol0 + ZC) {
          v = *reinterpret_cast<const float4*>(a.dout + row * H + c * 16 + 4 * g);
          if (a.mask_in) {
            v = mask4(v, mk, 4 * c);
          } else if (a.out_act) {
            const float4 m =
                *reinterpret_cast<const float4*>(a.out_act + row * H + c * 16 + 4 * g);
            v.x = m.x > 0.f ? v.x : 0.f; v.y = m.y > 0.f ? v.y : 0.f;
            v.z = m.z > 0.f ? v.z : 0.f; v.w = m.w > 0.f ? v.w : 0.f;
          }
        }
        z[c] = v;
      }
    };
    float4 dbacc[HC], zc[HC], zn[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) dbacc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    load_dz(0, zc);
    const float* wt_r = wt + i * LWT + 4 * g;
    for (int64_t it = 0; it <= n_my; ++it) {
      if (it < n_my) {
        // dz tile element (r, c) lives at r * LZ + (c ^ (((r >> 2) & 3) << 2)): the float4 writes
        // here (lane (i, g): row 16 zrow + i, 16-B slot g of each chunk) and the b32 column reads of
        // the X waves (lane (i, g): row 4 s + g, column 16 J + i) both hit 64 distinct banks
        float* dz_w = dzb + (it & 1) * T * LZ + (zrow * 16 + i) * LZ + 4 * (g ^ ((i >> 2) & 3));
        if (a.dz_out) {
          const int64_t row = (blockIdx.x + it * gridDim.x) * T + zrow * 16 + i;
          if (row < a.n) {
#pragma unroll
            for (int c = 0; c < HC; ++c)
              if (c >= zcol0 && c < zcol0 + ZC)
                *reinterpret_cast<float4*>(a.dz_out + row * H + c * 16 + 4 * g) = zc[c];
          }
        }
#pragma unroll
        for (int c = 0; c < HC; ++c) {
          if (c >= zcol0 && c < zcol0 + ZC) *reinterpret_cast<float4*>(dz_w + c * 16) = zc[c];
          dbacc[c].x += zc[c].x; dbacc[c].y += zc[c].y;
          dbacc[c].z += zc[c].z; dbacc[c].w += zc[c].w;
        }
        load_dz(it + 1, zn);
        if (DX) {
          const int64_t row = (blockIdx.x + it * gridDim.x) * T + zrow * 16 + i;
#pragma unroll
          for (int ct = 0; ct < KC; ct += 2) {
            f32x4 o0 = f32x4{0.f, 0.f, 0.f, 0.f}, o1 = o0;
#pragma unroll
            for (int c = 0; c < HC; ++c) {
              const float4 b0 = *reinterpret_cast<const float4*>(wt_r + ct * 16 * LWT + c * 16);
              const float4 b1 =
                  *reinterpret_cast<const float4*>(wt_r + (ct + 1) * 16 * LWT + c * 16);
              o0 = mfma4(b0.x, zc[c].x, o0); o1 = mfma4(b1.x, zc[c].x, o1);
              o0 = mfma4(b0.y, zc[c].y, o0); o1 = mfma4(b1.y, zc[c].y, o1);
              o0 = mfma4(b0.z, zc[c].z, o0); o1 = mfma4(b1.z, zc[c].z, o1);
              o0 = mfma4(b0.w, zc[c].w, o0); o1 = mfma4(b1.w, zc[c].w, o1);
            }
            if (row < a.n) {
#pragma unroll
              for (int h2 = 0; h2 < 2; ++h2) {
                float* dx = tab.dx[ct + h2];
                if (dx) {
                  const f32x4 o = h2 ? o1 : o0;
                  store_dx4(dx + row * tab.ld[ct + h2] + tab.col[ct + h2] + 4 * g,
                            (tab.dx_acc >> (ct + h2)) & 1u, o[0], o[1], o[2], o[3]);
                }
              }
            }
          }
        }
#pragma unroll
        for (int c = 0; c < HC; ++c) zc[c] = zn[c];
      }
      __syncthreads();
    }
    // bias: reduce over i (16 lanes), then over the 4 dz waves through LDS (fixed order)
    float* red = xsb;   // X buffers are idle after the final barrier of the X waves below
    __syncthreads();
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      float4 v = dbacc[c];
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) {
        v.x += __shfl_xor(v.x, m, 64); v.y += __shfl_xor(v.y, m, 64);
        v.z += __shfl_xor(v.z, m, 64); v.w += __shfl_xor(v.w, m, 64);
      }
      if (i == 0) *reinterpret_cast<float4*>(red + w4 * H + c * 16 + 4 * g) = v;
    }
    __syncthreads();
  } else {
    constexpr int XR = 256 / (K / 4);
    const int t4 = threadIdx.x - 256;
    const int xq_col = (t4 % (K / 4)) * 4, xq_row0 = t4 / (K / 4);
    const int xc = xq_col / 16;
    const float* xseg = tab.x[xc] + tab.col[xc] + (xq_col % 16);
    const int xld = tab.ld[xc];
    auto load_x = [&](int64_t it, float4 (&x)[XQ]) {
      const int64_t r0 = (blockIdx.x + it * gridDim.x) * T;
#pragma unroll
      for (int q = 0; q < XQ; ++q) {
        const int64_t row = r0 + xq_row0 + q * XR;
        x[q] = (it < n_my && row < a.n) ? *reinterpret_cast<const float4*>(xseg + row * xld)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    f32x4 wacc[JT][KC];
#pragma unroll
    for (int jt = 0; jt < JT; ++jt)
#pragma unroll
      for (int kt = 0; kt < KC; ++kt) wacc[jt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 xp[XQ];
    load_x(0, xp);
    for (int64_t it = 0; it <= n_my; ++it) {
      if (it < n_my) {
        float* xs_w = xsb + (it & 1) * T * LX + xq_row0 * LX + xq_col;
#pragma unroll
        for (int q = 0; q < XQ; ++q) *reinterpret_cast<float4*>(xs_w + q * XR * LX) = xp[q];
        load_x(it + 1, xp);
      }
      if (it >= 1) {   // wgrad of tile it-1 (its dz / X buffers were completed last barrier)
        const int b = (it - 1) & 1;
        const float* dz_r = dzb + b * T * LZ + g * LZ + (w4 * JT) * 16;
        const float* xs_r = xsb + b * T * LX + g * LX + i;
#pragma unroll 4
        for (int s4 = 0; s4 < T / 4; ++s4) {
          float az[JT];
#pragma unroll
          for (int jt = 0; jt < JT; ++jt)
            az[jt] = dz_r[s4 * 4 * LZ + jt * 16 + (i ^ ((s4 & 3) << 2))];   // swizzled (above)
#pragma unroll
          for (int kt = 0; kt < KC; ++kt) {
            const float bx = xs_r[s4 * 4 * LX + kt * 16];
#pragma unroll
            for (int jt = 0; jt < JT; ++jt) wacc[jt][kt] = mfma4(az[jt], bx, wacc[jt][kt]);
          }
        }
      }
      __syncthreads();
    }
    constexpr int KEXT = K + 1;
    float* slab = a.slab + (int64_t)blockIdx.x * H * KEXT;
#pragma unroll
    for (int jt = 0; jt < JT; ++jt)
#pragma unroll
      for (int kt = 0; kt < KC; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          slab[(int64_t)((w4 * JT + jt) * 16 + 4 * g + r) * KEXT + kt * 16 + i] =
              wacc[jt][kt][r];
    __syncthreads();
    __syncthreads();
  }
  // both roles passed the same number of barriers (n_my + 1, then 2)
  if (threadIdx.x < H) {
    const float* red = xsb;
    a.slab[(int64_t)blockIdx.x * H * (K + 1) + (int64_t)threadIdx.x * (K + 1) + K] =
        ((red[threadIdx.x] + red[H + threadIdx.x]) + red[2 * H + threadIdx.x]) +
        red[3 * H + threadIdx.x];
  }
}

// Weight gradient alone, v5: dW = dz^T [X_0 .. X_{S-1}] and db = colsum(dz), dz = dout * [out > 0].
// Persistent 512-thread blocks; every wave stages a share of each T-row tile (masked dz and X,
// float4 loads issued one tile ahead into registers) into double-buffered LDS, one barrier per
// tile, and EVERY wave runs MFMAs on the tile (v4's wgrad-only variant left the four dz-loading
// waves without MFMA work: one MFMA wave per SIMD).  Wave w owns 2 j-tiles x KW k-tiles of the
// [H][K] output: per 4-row k-step 2 + KW b32 LDS reads feed 2 KW independent MFMAs.  Row strides
// H+16 / K+16 keep the b32 reads conflict-free.  The block's partial dW/db goes to its slab
// (k_wgrad_reduce sums the slabs in block order: deterministic).
template <int H, int K, int T>
__global__ void __launch_bounds__(512) k_linear_wgrad_v5(const LinArgs a, const ChunkTab tab,
                                                         int64_t n_tiles) {
  constexpr int HC = H / 16, KC = K / 16;
  constexpr int JG = HC / 2;                 // j-tile pairs
  constexpr int KG = 8 / JG;                 // k groups per j pair (8 waves)
  constexpr int KW = KC / KG;                // k tiles per wave
  static_assert(JG * KG == 8 && KW * KG == KC, "wave split");
  constexpr int LZ = H + 16, LX = K + 16;
  constexpr int ZQ = T * H / 4 / 512;        // dz float4 per thread per tile
  constexpr int XQ = T * K / 4 / 512;        // X float4 per thread per tile
  static_assert(ZQ >= 1 && XQ >= 1, "tile too small for 512 threads");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* dzb = smem;                         // 2 x [T][LZ]
  float* xsb = dzb + 2 * T * LZ;             // 2 x [T][LX]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int jt0 = 2 * (wave / KG), kt0 = (wave % KG) * KW;
  // fixed staging columns per thread (H/4 and K/4 divide 512)
  const int zc4 = threadIdx.x % (H / 4), zr0 = threadIdx.x / (H / 4);
  constexpr int ZR = 512 / (H / 4);          // rows apart between a thread's dz float4
  const int xk4 = threadIdx.x % (K / 4), xr0 = threadIdx.x / (K / 4);
  constexpr int XR = 512 / (K / 4);
  const int xc = xk4 / 4;
  const float* xseg = tab.x[xc] + tab.col[xc] + 4 * (xk4 % 4);
  const int xld = tab.ld[xc];
  const bool bits = a.mask_in != nullptr;
  const bool masked = !bits && a.out_act != nullptr;
  const int64_t n_my = (n_tiles - blockIdx.x + gridDim.x - 1) / gridDim.x;
  const int64_t last = a.n - 1;
  float4 zp[ZQ], mp[ZQ], xp[XQ];
  uint32_t bp[ZQ];
  const int bshift = 4 * (zc4 >> 2);        // columns 4 zc4 .. +3: chunk zc4/4, lane group zc4%4
  auto issue = [&](int64_t it) {
    const int64_t r0 = (blockIdx.x + it * gridDim.x) * T;
#pragma unroll
    for (int q = 0; q < ZQ; ++q) {
      const int64_t row = min<int64_t>(r0 + zr0 + q * ZR, last);
      zp[q] = *reinterpret_cast<const float4*>(a.dout + row * H + 4 * zc4);
      if (bits) bp[q] = a.mask_in[row * 4 + (zc4 & 3)];
      if (masked) mp[q] = *reinterpret_cast<const float4*>(a.out_act + row * H + 4 * zc4);
    }
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int64_t row = min<int64_t>(r0 + xr0 + q * XR, last);
      xp[q] = *reinterpret_cast<const float4*>(xseg + row * xld);
    }
  };
  f32x4 acc[2][KW];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int k = 0; k < KW; ++k) acc[j][k] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 dbacc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n_my > 0) issue(0);
  for (int64_t it = 0; it < n_my; ++it) {
    const int b = it & 1;
    const int64_t r0 = (blockIdx.x + it * gridDim.x) * T;
    float* dz_w = dzb + b * T * LZ;
    float* xs_w = xsb + b * T * LX;
#pragma unroll
    for (int q = 0; q < ZQ; ++q) {
      const int r = zr0 + q * ZR;
      float4 v = zp[q];
      if (bits) v = mask4(v, bp[q], bshift);
      if (masked) {
        v.x = mp[q].x > 0.f ? v.x : 0.f; v.y = mp[q].y > 0.f ? v.y : 0.f;
        v.z = mp[q].z > 0.f ? v.z : 0.f; v.w = mp[q].w > 0.f ? v.w : 0.f;
      }
      if (r0 + r >= a.n) v = make_float4(0.f, 0.f, 0.f, 0.f);   // clamped rows contribute 0
      dbacc.x += v.x; dbacc.y += v.y; dbacc.z += v.z; dbacc.w += v.w;
      *reinterpret_cast<float4*>(dz_w + r * LZ + 4 * zc4) = v;
    }
#pragma unroll
    for (int q = 0; q < XQ; ++q)
      *reinterpret_cast<float4*>(xs_w + (xr0 + q * XR) * LX + 4 * xk4) = xp[q];
    if (it + 1 < n_my) issue(it + 1);
    __syncthreads();
    const float* dz_r = dz_w + g * LZ + jt0 * 16 + i;
    const float* xs_r = xs_w + g * LX + kt0 * 16 + i;
#pragma unroll 4
    for (int s4 = 0; s4 < T / 4; ++s4) {
      const float a0 = dz_r[s4 * 4 * LZ], a1 = dz_r[s4 * 4 * LZ + 16];
#pragma unroll
      for (int k = 0; k < KW; ++k) {
        const float bx = xs_r[s4 * 4 * LX + k * 16];
        acc[0][k] = mfma4(a0, bx, acc[0][k]);
        acc[1][k] = mfma4(a1, bx, acc[1][k]);
      }
    }
  }
  constexpr int KEXT = K + 1;
  float* slab = a.slab + (int64_t)blockIdx.x * H * KEXT;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int k = 0; k < KW; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        slab[(int64_t)((jt0 + j) * 16 + 4 * g + r) * KEXT + (kt0 + k) * 16 + i] = acc[j][k][r];
  // db: thread partials (fixed column 4*zc4) reduced through LDS in a fixed order
  __syncthreads();
  float4* red = reinterpret_cast<float4*>(smem);
  red[threadIdx.x] = dbacc;
  __syncthreads();
  if (threadIdx.x < H / 4) {
    float4 t = red[threadIdx.x];
    for (int m = threadIdx.x + H / 4; m < 512; m += H / 4) {
      const float4 u = red[m];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    const int c = threadIdx.x * 4;
    slab[(int64_t)(c + 0) * KEXT + K] = t.x;
    slab[(int64_t)(c + 1) * KEXT + K] = t.y;
    slab[(int64_t)(c + 2) * KEXT + K] = t.z;
    slab[(int64_t)(c + 3) * KEXT + K] = t.w;
  }
}

static size_t wgrad5_lds(int h, int k, int t) {
  return std::max<size_t>(((size_t)2 * t * (h + 16) + (size_t)2 * t * (k + 16)) * 4, 512 * 16);
}

static size_t v4_bwd_lds(int h, int k, bool dx, int t = 64) {
  return ((dx ? (size_t)k * (h + 8) : 0) + (size_t)2 * t * (h + 16) + (size_t)2 * t * (k + 16)) *
         4;
}

// dgrad alone, persistent: dX = (dout * [out > 0]) W with W^T staged in LDS once per block
// ([K][H+8], conflict-free b128 fragments); each of the 8 waves streams its own 16-row tiles with
// the next tile's masked dz fragments in flight, and computes dX^T = W^T dz^T so that every lane
// stores float4 runs of its row.  Used with the wgrad-only kernel when the fused backward's LDS
// (W^T + two dz and X tiles) does not fit: K = 256, or H = 128 with K = 128.
template <int H, int K>
__global__ void __launch_bounds__(512) k_linear_dgrad_v4(const LinArgs a, const ChunkTab tab,
                                                         int64_t n_tiles) {
  constexpr int HC = H / 16, KC = K / 16, LWT = H + 8;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* wt = smem;   // [K][LWT]
  for (int idx = threadIdx.x; idx < H * K; idx += 512) {
    const int j = idx / K, k = idx % K;
    wt[k * LWT + j] = a.w[(int64_t)j * K + k];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int64_t nw = (int64_t)gridDim.x * 8;
  auto load_dz = [&](int64_t t, float4 (&z)[HC]) {
    const int64_t row = t * 16 + i;
    const uint32_t mk = a.mask_in && row < a.n ? a.mask_in[row * 4 + g] : 0u;
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < a.n) {
        v = *reinterpret_cast<const float4*>(a.dout + row * H + c * 16 + 4 * g);
        if (a.mask_in) {
          v = mask4(v, mk, 4 * c);
        } else if (a.out_act) {
          const float4 m = *reinterpret_cast<const float4*>(a.out_act + row * H + c * 16 + 4 * g);
          v.x = m.x > 0.f ? v.x : 0.f; v.y = m.y > 0.f ? v.y : 0.f;
          v.z = m.z > 0.f ? v.z : 0.f; v.w = m.w > 0.f ? v.w : 0.f;
        }
      }
      z[c] = v;
    }
  };
  int64_t t = (int64_t)blockIdx.x * 8 + wave;
  float4 zc[HC], zn[HC];
  if (t < n_tiles) load_dz(t, zc);
  __syncthreads();
  const int wr0 = i * LWT + 4 * g;
  for (; t < n_tiles; t += nw) {
    if (t + nw < n_tiles) load_dz(t + nw, zn);
    int wo = wr0;
    asm volatile("" : "+v"(wo));   // keep W^T fragments as per-tile LDS reads (see fwd v4)
    const float* wt_r = wt + wo;
    const int64_t row = t * 16 + i;
    if (a.dz_out && row < a.n) {
#pragma unroll
      for (int c = 0; c < HC; ++c)
        *reinterpret_cast<float4*>(a.dz_out + row * H + c * 16 + 4 * g) = zc[c];
    }
#pragma unroll
    for (int ct = 0; ct < KC; ct += 2) {
      f32x4 o0 = f32x4{0.f, 0.f, 0.f, 0.f}, o1 = o0;
#pragma unroll
      for (int c = 0; c < HC; ++c) {
        const float4 b0 = *reinterpret_cast<const float4*>(wt_r + ct * 16 * LWT + c * 16);
        const float4 b1 = *reinterpret_cast<const float4*>(wt_r + (ct + 1) * 16 * LWT + c * 16);
        o0 = mfma4(b0.x, zc[c].x, o0); o1 = mfma4(b1.x, zc[c].x, o1);
        o0 = mfma4(b0.y, zc[c].y, o0); o1 = mfma4(b1.y, zc[c].y, o1);
        o0 = mfma4(b0.z, zc[c].z, o0); o1 = mfma4(b1.z, zc[c].z, o1);
        o0 = mfma4(b0.w, zc[c].w, o0); o1 = mfma4(b1.w, zc[c].w, o1);
      }
      if (row < a.n) {
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          float* dx = tab.dx[ct + h2];
          if (dx) {
            const f32x4 o = h2 ? o1 : o0;
            store_dx4(dx + row * tab.ld[ct + h2] + tab.col[ct + h2] + 4 * g,
                      (tab.dx_acc >> (ct + h2)) & 1u, o[0], o[1], o[2], o[3]);
          }
        }
      }
    }
#pragma unroll
    for (int c = 0; c < HC; ++c) zc[c] = zn[c];
  }
}

static size_t dgrad4_lds(int h, int k) { return (size_t)k * (h + 8) * 4; }

// dgrad v5: v4's tiling and W^T image, reorganised for 2 waves per SIMD: G column
// tiles in flight (G independent accumulators, k-step-major), W^T fragments read one k-sweep ahead
// (across column-group boundaries too), and the next tile's raw dout / out fragments held as
// loaded — the ReLU mask is applied when the tile becomes current, so no load is waited for at
// issue.  Rows past the end are clamped (loaded, never stored).
template <int H, int K>
__global__ void __launch_bounds__(512, 2) k_linear_dgrad_v5(const LinArgs a, const ChunkTab tab,
                                                            int64_t n_tiles) {
  constexpr int HC = H / 16, KC = K / 16, LWT = H + 8;
  constexpr int G = KC < 8 ? KC : 8, NG = KC / G;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* wt = smem;   // [K][LWT]
  for (int idx = threadIdx.x; idx < H * K; idx += 512) {
    const int j = idx / K, k = idx % K;
    wt[k * LWT + j] = a.w[(int64_t)j * K + k];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int64_t nw = (int64_t)gridDim.x * 8;
  const int64_t last = a.n - 1;
  const bool bits = a.mask_in != nullptr;
  const bool masked = !bits && a.out_act != nullptr;
  float4 zr[HC], mr[HC];
  uint32_t mk = 0u;
  auto issue = [&](int64_t t) {
    const int64_t row = min<int64_t>(t * 16 + i, last);
    if (bits) mk = a.mask_in[row * 4 + g];
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      zr[c] = *reinterpret_cast<const float4*>(a.dout + row * H + c * 16 + 4 * g);
      if (masked) mr[c] = *reinterpret_cast<const float4*>(a.out_act + row * H + c * 16 + 4 * g);
    }
  };
  int64_t t = (int64_t)blockIdx.x * 8 + wave;
  if (t < n_tiles) issue(t);
  __syncthreads();
  const int wr0 = i * LWT + 4 * g;
  for (; t < n_tiles; t += nw) {
    float4 zc[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      zc[c] = zr[c];
      if (bits) zc[c] = mask4(zc[c], mk, 4 * c);
      if (masked) {
        zc[c].x = mr[c].x > 0.f ? zc[c].x : 0.f; zc[c].y = mr[c].y > 0.f ? zc[c].y : 0.f;
        zc[c].z = mr[c].z > 0.f ? zc[c].z : 0.f; zc[c].w = mr[c].w > 0.f ? zc[c].w : 0.f;
      }
    }
    issue(t + nw < n_tiles ? t + nw : t);
    int wo = wr0;
    asm volatile("" : "+v"(wo));   // keep W^T fragments as per-tile LDS reads (see fwd v4)
    const float* wt_r = wt + wo;
    const int64_t row = t * 16 + i;
    if (a.dz_out && row < a.n) {
#pragma unroll
      for (int c = 0; c < HC; ++c)
        *reinterpret_cast<float4*>(a.dz_out + row * H + c * 16 + 4 * g) = zc[c];
    }
    float4 bw[G];
#pragma unroll
    for (int j = 0; j < G; ++j) bw[j] = *reinterpret_cast<const float4*>(wt_r + j * 16 * LWT);
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
      f32x4 o[G];
#pragma unroll
      for (int j = 0; j < G; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < HC; ++c) {
#pragma unroll
        for (int j = 0; j < G; ++j) o[j] = mfma4(bw[j].x, zc[c].x, o[j]);
#pragma unroll
        for (int j = 0; j < G; ++j) o[j] = mfma4(bw[j].y, zc[c].y, o[j]);
#pragma unroll
        for (int j = 0; j < G; ++j) o[j] = mfma4(bw[j].z, zc[c].z, o[j]);
#pragma unroll
        for (int j = 0; j < G; ++j) {
          o[j] = mfma4(bw[j].w, zc[c].w, o[j]);
          if (c + 1 < HC)
            bw[j] = *reinterpret_cast<const float4*>(wt_r + (gi * G + j) * 16 * LWT + (c + 1) * 16);
          else if (gi + 1 < NG)
            bw[j] = *reinterpret_cast<const float4*>(wt_r + ((gi + 1) * G + j) * 16 * LWT);
        }
      }
      if (row < a.n) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
          const int ct = gi * G + j;
          float* dx = tab.dx[ct];
          if (dx)
            store_dx4(dx + row * tab.ld[ct] + tab.col[ct] + 4 * g, (tab.dx_acc >> ct) & 1u,
                      o[j][0], o[j][1], o[j][2], o[j][3]);
        }
      }
    }
  }
}



// ReLU mask bits from a finished output (forward shapes without a persistent kernel), in the
// lane layout of mask4: one thread per (row, lane group g).
__global__ void k_relu_mask(const float* out, int64_t n, int32_t h, uint32_t* mask) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * 4) return;
  const int64_t row = idx >> 2;
  const int g = (int)(idx & 3);
  uint32_t m = 0;
  for (int c = 0; c < h / 16; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      m |= (out[row * h + 16 * c + 4 * g + e] > 0.f ? 1u : 0u) << (4 * c + e);
  mask[idx] = m;
}

// the persistent forward also takes K = 256 (W: H*(K+8)*4 <= 135 KB of LDS, one block per CU)
static bool fwd4_ok(const LinArgs& a, bool vec) {
  if (!vec || !(a.h == 64 || a.h == 128) ||
      !(a.k_total == 64 || a.k_total == 128 || a.k_total == 256))
    return false;
  for (int s = 0; s < a.n_seg; ++s)
    if (a.seg[s].k % 16) return false;
  return true;
}

// the chunks of columns [c0, c0 + kp) of the concatenated input (every segment a multiple of 16)
static ChunkTab chunk_table_range(const LinArgs& a, int c0, int kp) {
  ChunkTab t{};
  for (int c = 0; c < kp / 16 && c < kMaxChunks; ++c) {
    const int k = c0 + c * 16;
    int s = 0;
    while (s + 1 < a.n_seg && k >= a.seg[s].off + a.seg[s].k) ++s;
    t.x[c] = a.seg[s].x;
    t.dx[c] = a.seg[s].dx;
    if ((a.dx_acc >> s) & 1u) t.dx_acc |= 1u << c;
    t.ld[c] = a.seg[s].k;
    t.col[c] = k - a.seg[s].off;
  }
  return t;
}
static ChunkTab chunk_table(const LinArgs& a) { return chunk_table_range(a, 0, a.k_total); }

// K = 384 / 512 at H = 128 (the sampled blocks' [aggr_1 | aggr_2 | root] at d = 128) on the
// split-once kernels as two column blocks, [0, 256) and [256, K): the forward's second launch
// adds the first one's output rows (its own `add`, read before the same block stores them)
// and applies the bias, activation and mask; the backward runs each block's dgrad / wgrad into
// its columns of one shared [G][h][K + 1] slab, reduced once.  Replaces the f32-input general
// kernels there (51 / 65 us per launch at cfg5's ~17k rows).
// Blocks of every size take it: at cfg5's inner blocks (2-3k rows) the general kernels measured
// the same time one destination type at a time (0.680 vs 0.677 ms per batch, 4 launches fewer),
// but with both types paired into one launch per column block (hgnn_linear_fwd_multi) the split
// kernels are faster: 0.603 / 0.604 vs 0.622 / 0.621 ms per batch, 22 vs 24 launches
// (profiles/r6_wide_min_ab.txt).
static bool xs_wide_ok(const LinArgs& a, bool vec) {
  if (!vec || a.h != 128 || a.k_total <= 256 || a.k_total > 512 || a.k_total % 128 != 0)
    return false;
  for (int s = 0; s < a.n_seg; ++s)
    if (a.seg[s].k % 16) return false;
  return x6_enabled();
}

// The two column blocks pass the first one's partial rows through `out`, so out must not alias
// an input segment (or `add`) on this path; such a call goes to the general kernels instead
// (ADVICE r5).  Byte ranges of n rows each.
static bool out_overlaps_inputs(const LinArgs& a) {
  const uintptr_t o0 = reinterpret_cast<uintptr_t>(a.out);
  const uintptr_t o1 = o0 + (uintptr_t)a.n * a.h * 4;
  auto hit = [&](const void* p, int64_t row_floats) {
    const uintptr_t p0 = reinterpret_cast<uintptr_t>(p), p1 = p0 + (uintptr_t)a.n * row_floats * 4;
    return p && p0 < o1 && o0 < p1;
  };
  for (int s = 0; s < a.n_seg; ++s)
    if (hit(a.seg[s].x, a.seg[s].k)) return true;
  return hit(a.add, a.h);
}

static int xs_fwd_wide(const LinArgs& a, hipStream_t stream) {
  LinArgs A = a;
  A.k_total = 256;
  A.bias = nullptr;
  A.relu = 0;
  A.mask_out = nullptr;   // A.add: the caller's rows, if any
  if (int rc = xs_linear_fwd(A, chunk_table_range(a, 0, 256), stream)) return rc;
  LinArgs B = a;
  B.k_total = a.k_total - 256;
  B.w = a.w + 256;
  B.add = a.out;
  return xs_linear_fwd(B, chunk_table_range(a, 256, B.k_total), stream);
}

static int xs_bwd_wide(const LinArgs& a, float* dw, float* db, void* ws, size_t ws_bytes,
                       hipStream_t stream) {
  const bool wg = dw || db;
  const int K = a.k_total;
  int G = 0;
  if (wg) {   // one slab [G][h][K + 1] for both column blocks, one reduce
    const size_t need = (size_t)xs_bwd_grid(a.n) * a.h * (K + 1) * 4;
    if (!ws || ws_bytes < need) return fail(HGNN_E_WS, "linear_bwd: workspace too small");
  }
  for (int part = 0; part < 2; ++part) {
    const int c0 = part ? 256 : 0, kp = part ? a.k_total - 256 : 256;
    LinArgs P = a;
    P.k_total = kp;
    P.w = a.w + c0;
    P.dz_out = nullptr;
    const ChunkTab tab = chunk_table_range(a, c0, kp);
    bool pdx = false;
    for (int c = 0; c < kp / 16; ++c) pdx |= tab.dx[c] != nullptr;
    P.slab = wg ? static_cast<float*>(ws) : nullptr;
    P.slab_ld = K + 1;
    P.slab_c0 = c0;
    if (pdx || wg) {
      if (int rc = xs_linear_bwd(P, tab, pdx, &G, stream)) return rc;
    }
  }
  if (!wg) return HGNN_OK;
  const int64_t total = (int64_t)a.h * (K + 1);
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)cdiv(total, 64)), dim3(1024), 0, stream,
                     static_cast<const float*>(ws), (int64_t)G, a.h, K + 1, dw, db, K);
  return check_launch("k_wgrad_reduce");
}

// ---- two jobs per launch (the two destination types of a sampled layer) ----
// Both jobs on the K = 384 / 512 split path with the same K: each column block is one launch for
// both (k_lin_fwd_xs2 / k_lin_bwd_xs2) and the backward's two slabs one reduce (k_wgrad_reduce2),
// 5 launches where job by job takes 10.  HGNN_K3_PAIR=0: job by job.
static bool pair_enabled() {
  static const bool v = !getenv("HGNN_K3_PAIR") || atoi(getenv("HGNN_K3_PAIR")) != 0;
  return v;
}

// byte range [p, p + bytes) against [q, q + qbytes)
static bool ranges_overlap(const void* p, size_t bytes, const void* q, size_t qbytes) {
  if (!p || !q) return false;
  const uintptr_t p0 = reinterpret_cast<uintptr_t>(p), q0 = reinterpret_cast<uintptr_t>(q);
  return p0 < q0 + qbytes && q0 < p0 + bytes;
}

// what job `a` reads, against a range job `b` writes (the jobs run side by side in a pair)
static bool reads_overlap(const LinArgs& a, const void* p, size_t bytes) {
  const size_t rows = (size_t)a.n * 4;
  for (int s = 0; s < a.n_seg; ++s)
    if (ranges_overlap(a.seg[s].x, rows * a.seg[s].k, p, bytes) ||
        ranges_overlap(a.seg[s].dx, rows * a.seg[s].k, p, bytes))
      return true;
  return ranges_overlap(a.add, rows * a.h, p, bytes) || ranges_overlap(a.dout, rows * a.h, p, bytes) ||
         ranges_overlap(a.out_act, rows * a.h, p, bytes) ||
         ranges_overlap(a.mask_in, rows * 4, p, bytes) ||
         ranges_overlap(a.out, rows * a.h, p, bytes);
}

static bool writes_hit(const LinArgs& w, const LinArgs& r) {
  const size_t rows = (size_t)w.n * 4;
  if (reads_overlap(r, w.out, rows * w.h) || reads_overlap(r, w.mask_out, rows * 4)) return true;
  for (int s = 0; s < w.n_seg; ++s)
    if (reads_overlap(r, w.seg[s].dx, rows * w.seg[s].k)) return true;
  return false;
}

static int xs_fwd_wide2(const LinArgs (&a)[2], hipStream_t stream) {
  LinArgs A[2], B[2];
  ChunkTab TA[2], TB[2];
  for (int j = 0; j < 2; ++j) {
    A[j] = a[j];
    A[j].k_total = 256;
    A[j].bias = nullptr;
    A[j].relu = 0;
    A[j].mask_out = nullptr;
    TA[j] = chunk_table_range(a[j], 0, 256);
    B[j] = a[j];
    B[j].k_total = a[j].k_total - 256;
    B[j].w = a[j].w + 256;
    B[j].add = a[j].out;
    TB[j] = chunk_table_range(a[j], 256, B[j].k_total);
  }
  if (int rc = xs_linear_fwd2(A, TA, stream)) return rc;
  return xs_linear_fwd2(B, TB, stream);
}

// the backward's column blocks of both jobs; false (nothing launched) when their variants differ
static bool xs_bwd_parts(const LinArgs (&a)[2], float* const (&slab)[2], LinArgs (&P)[2][2],
                         ChunkTab (&T)[2][2], bool (&pdx)[2]) {
  for (int part = 0; part < 2; ++part) {
    int cls[2];
    bool d[2];
    for (int j = 0; j < 2; ++j) {
      const int c0 = part ? 256 : 0, kp = part ? a[j].k_total - 256 : 256;
      LinArgs& p = P[part][j];
      p = a[j];
      p.k_total = kp;
      p.w = a[j].w + c0;
      p.dz_out = nullptr;
      T[part][j] = chunk_table_range(a[j], c0, kp);
      d[j] = false;
      for (int c = 0; c < kp / 16; ++c) d[j] |= T[part][j].dx[c] != nullptr;
      p.slab = slab[j];
      p.slab_ld = a[j].k_total + 1;
      p.slab_c0 = c0;
      cls[j] = xs_bwd_class(p, T[part][j], d[j]);
    }
    if (cls[0] != cls[1]) return false;
    pdx[part] = d[0];
  }
  return true;
}

static int xs_bwd_wide2(LinArgs (&P)[2][2], ChunkTab (&T)[2][2], const bool (&pdx)[2],
                        float* const (&dw)[2], float* const (&db)[2], hipStream_t stream) {
  const bool wg = P[0][0].slab != nullptr;
  int G[2] = {0, 0};
  for (int part = 0; part < 2; ++part) {
    if (pdx[part] || wg) {
      LinArgs pa[2] = {P[part][0], P[part][1]};
      ChunkTab pt[2] = {T[part][0], T[part][1]};
      if (int rc = xs_linear_bwd2(pa, pt, pdx[part], G, stream)) return rc;
    }
  }
  if (!wg) return HGNN_OK;
  const int K = P[0][0].slab_ld - 1, h = P[0][0].h;
  ReducePair r;
  const int64_t total = (int64_t)h * (K + 1);
  for (int j = 0; j < 2; ++j) {
    r.slab[j] = P[0][j].slab;
    r.nb[j] = G[j];
    r.dw[j] = dw[j];
    r.db[j] = db[j];
  }
  r.nblk0 = cdiv(total, 64);
  r.h = h;
  r.kext = K + 1;
  r.ldd = K;
  hipLaunchKernelGGL(k_wgrad_reduce2, dim3((unsigned)(2 * r.nblk0)), dim3(1024), 0, stream, r);
  return check_launch("k_wgrad_reduce2");
}

// every 8 consecutive 16-column chunks one 128-column segment (x_chunk<true>'s addressing)
static bool chunks_in_segments_of_8(const ChunkTab& tab, int k_total) {
  for (int c = 0; c < k_total / 16; ++c) {
    const int s = c & ~7;
    if (tab.x[c] != tab.x[s] || tab.ld[c] != tab.ld[s] || tab.col[c] != tab.col[s] + (c & 7) * 16)
      return false;
  }
  return true;
}

static int fill_args(LinArgs& a, int32_t n_seg, const float* const* xs, const int32_t* ks,
                     float* const* dxs, int64_t n_rows, const float* w, int32_t h, bool* vec) {
  if (n_seg < 1 || n_seg > HGNN_MAX_SEG) return fail(HGNN_E_ARG, "linear: n_seg=%d", n_seg);
  if (h < 1 || n_rows < 0 || !w || !xs || !ks) return fail(HGNN_E_ARG, "linear: bad arguments");
  a.n_seg = n_seg;
  a.k_total = 0;
  *vec = (h % 4 == 0);
  for (int s = 0; s < n_seg; ++s) {
    if (ks[s] < 1 || (n_rows > 0 && !xs[s])) return fail(HGNN_E_ARG, "linear: segment %d", s);
    a.seg[s].x = xs[s];
    a.seg[s].dx = dxs ? dxs[s] : nullptr;
    a.seg[s].k = ks[s];
    a.seg[s].off = a.k_total;
    a.k_total += ks[s];
    *vec = *vec && ks[s] % 4 == 0 && (reinterpret_cast<uintptr_t>(xs[s]) % 16 == 0);
  }
  *vec = *vec && reinterpret_cast<uintptr_t>(w) % 16 == 0;
  a.w = w;
  a.ldw = a.k_total;
  a.n = n_rows;
  a.h = h;
  return HGNN_OK;
}

// a forward job's arguments as hgnn_linear_fwd_mask (add = NULL) fills them, and whether that call
// would take the K = 384 / 512 split path; false on any argument the call itself would refuse
static bool fwd_wide_job(LinArgs& a, int32_t n_seg, const float* const* xs, const int32_t* ks,
                         int64_t n_rows, const float* w, int32_t h, const float* bias,
                         int32_t relu, float* out, uint32_t* mask) {
  a = LinArgs{};
  bool vec;
  if (fill_args(a, n_seg, xs, ks, nullptr, n_rows, w, h, &vec) != HGNN_OK) return false;
  if (mask && (!relu || h % 16 != 0 || h > 128)) return false;
  if (n_rows == 0 || !out) return false;
  a.bias = bias;
  a.out = out;
  a.relu = relu;
  a.mask_out = mask;
  return xs_wide_ok(a, vec && reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                           reinterpret_cast<uintptr_t>(bias) % 16 == 0) &&
         !out_overlaps_inputs(a);
}

// the same for a backward job (hgnn_linear_bwd_ex with dz_out = NULL)
static bool bwd_wide_job(LinArgs& a, int32_t n_seg, const float* const* xs, const int32_t* ks,
                         int64_t n_rows, const float* w, int32_t h, const float* dout,
                         const float* out, const uint32_t* mask, float* const* dxs,
                         uint32_t dx_accumulate, bool wg, bool have_ws) {
  a = LinArgs{};
  bool vec;
  if (fill_args(a, n_seg, xs, ks, dxs, n_rows, w, h, &vec) != HGNN_OK) return false;
  if ((dx_accumulate >> n_seg) || !dout || n_rows == 0) return false;
  if (mask && (!out || h % 16 != 0 || h > 128)) return false;
  a.dx_acc = dx_accumulate;
  a.dout = dout;
  a.out_act = out;
  a.mask_in = mask;
  vec = vec && reinterpret_cast<uintptr_t>(dout) % 16 == 0 &&
        (!out || reinterpret_cast<uintptr_t>(out) % 16 == 0);
  for (int s = 0; s < n_seg; ++s)
    vec = vec && (!a.seg[s].dx || reinterpret_cast<uintptr_t>(a.seg[s].dx) % 16 == 0);
  return xs_wide_ok(a, vec) && (have_ws || !wg);
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_linear_fwd_multi(int32_t n_jobs, const int32_t* n_seg, const float* const* xs,
                          const int32_t* ks, const int64_t* n_rows, const float* const* w,
                          int32_t h, const float* const* bias, const int32_t* relu,
                          float* const* out, uint32_t* const* mask, hgnn_stream_t stream_) {
  if (n_jobs < 0 || (n_jobs > 0 && (!n_seg || !xs || !ks || !n_rows || !w || !out)))
    return fail(HGNN_E_ARG, "linear_fwd_multi: bad arguments");
  for (int j = 0; j < n_jobs; ++j)
    if (n_seg[j] < 1 || n_seg[j] > HGNN_MAX_SEG)
      return fail(HGNN_E_ARG, "linear_fwd_multi: job %d has n_seg=%d", j, n_seg[j]);
  if (n_jobs == 2 && pair_enabled()) {
    LinArgs a[2];
    bool ok = true;
    for (int j = 0, o = 0; j < 2 && ok; o += n_seg[j], ++j)
      ok = fwd_wide_job(a[j], n_seg[j], xs + o, ks + o, n_rows[j], w[j], h, bias ? bias[j] : nullptr,
                        relu ? relu[j] : 0, out[j], mask ? mask[j] : nullptr);
    if (ok && a[0].k_total == a[1].k_total && !writes_hit(a[0], a[1]) && !writes_hit(a[1], a[0]))
      return xs_fwd_wide2(a, as_stream(stream_));
  }
  for (int j = 0, o = 0; j < n_jobs; o += n_seg[j], ++j)
    if (int rc = hgnn_linear_fwd_mask(n_seg[j], xs + o, ks + o, n_rows[j], w[j], h,
                                      bias ? bias[j] : nullptr, nullptr, relu ? relu[j] : 0,
                                      out[j], mask ? mask[j] : nullptr, stream_))
      return rc;
  return HGNN_OK;
}

size_t hgnn_linear_bwd_multi_ws_bytes(int32_t n_jobs, const int64_t* n_rows,
                                      const int32_t* k_total, int32_t h) {
  size_t total = 0;
  for (int j = 0; j < n_jobs; ++j) total += hgnn_linear_bwd_ws_bytes(n_rows[j], k_total[j], h);
  return total;
}

int hgnn_linear_bwd_multi(int32_t n_jobs, const int32_t* n_seg, const float* const* xs,
                          const int32_t* ks, const int64_t* n_rows, const float* const* w,
                          int32_t h, const float* const* dout, const float* const* out,
                          const uint32_t* const* mask, float* const* dxs,
                          const uint32_t* dx_accumulate, float* const* dw, float* const* db,
                          void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  if (n_jobs < 0 || (n_jobs > 0 && (!n_seg || !xs || !ks || !n_rows || !w || !dout)))
    return fail(HGNN_E_ARG, "linear_bwd_multi: bad arguments");
  // job j's workspace: its hgnn_linear_bwd_ws_bytes, one after the other
  char* wsp[2] = {nullptr, nullptr};
  size_t wsb[2] = {0, 0};
  size_t off = 0;
  for (int j = 0, o = 0; j < n_jobs; o += n_seg[j], ++j) {
    if (n_seg[j] < 1 || n_seg[j] > HGNN_MAX_SEG)
      return fail(HGNN_E_ARG, "linear_bwd_multi: job %d has n_seg=%d", j, n_seg[j]);
    int32_t k = 0;
    for (int s = 0; s < n_seg[j]; ++s) k += ks[o + s];
    const size_t b = hgnn_linear_bwd_ws_bytes(n_rows[j], k, h);
    if (j < 2) { wsp[j] = ws ? static_cast<char*>(ws) + off : nullptr; wsb[j] = b; }
    off += b;
  }
  const bool any_w = [&] {
    for (int j = 0; j < n_jobs; ++j) if ((dw && dw[j]) || (db && db[j])) return true;
    return false;
  }();
  if (any_w && (!ws || ws_bytes < off)) return fail(HGNN_E_WS, "linear_bwd_multi: workspace too small");
  hipStream_t stream = as_stream(stream_);
  if (n_jobs == 2 && pair_enabled()) {
    LinArgs a[2];
    bool ok = true;
    for (int j = 0, o = 0; j < 2 && ok; o += n_seg[j], ++j) {
      const bool wg = (dw && dw[j]) || (db && db[j]);
      ok = bwd_wide_job(a[j], n_seg[j], xs + o, ks + o, n_rows[j], w[j], h, dout[j],
                        out ? out[j] : nullptr, mask ? mask[j] : nullptr, dxs ? dxs + o : nullptr,
                        dx_accumulate ? dx_accumulate[j] : 0u, wg, wsp[j] != nullptr);
      if (ok && wg) {
        const size_t need = (size_t)xs_bwd_grid(a[j].n) * h * (a[j].k_total + 1) * 4;
        ok = wsb[j] >= need;
      }
    }
    if (ok && a[0].k_total == a[1].k_total && !writes_hit(a[0], a[1]) && !writes_hit(a[1], a[0])) {
      float* slab[2];
      float* dwj[2];
      float* dbj[2];
      for (int j = 0; j < 2; ++j) {
        dwj[j] = dw ? dw[j] : nullptr;
        dbj[j] = db ? db[j] : nullptr;
        slab[j] = (dwj[j] || dbj[j]) ? reinterpret_cast<float*>(wsp[j]) : nullptr;
      }
      LinArgs P[2][2];
      ChunkTab T[2][2];
      bool pdx[2];
      if (xs_bwd_parts(a, slab, P, T, pdx)) return xs_bwd_wide2(P, T, pdx, dwj, dbj, stream);
    }
  }
  off = 0;
  for (int j = 0, o = 0; j < n_jobs; o += n_seg[j], ++j) {
    int32_t k = 0;
    for (int s = 0; s < n_seg[j]; ++s) k += ks[o + s];
    const size_t b = hgnn_linear_bwd_ws_bytes(n_rows[j], k, h);
    if (int rc = hgnn_linear_bwd_ex(n_seg[j], xs + o, ks + o, n_rows[j], w[j], h, dout[j],
                                    out ? out[j] : nullptr, mask ? mask[j] : nullptr,
                                    dxs ? dxs + o : nullptr, dx_accumulate ? dx_accumulate[j] : 0u,
                                    dw ? dw[j] : nullptr, db ? db[j] : nullptr, nullptr,
                                    ws ? static_cast<char*>(ws) + off : nullptr, ws ? b : 0,
                                    stream_))
      return rc;
    off += b;
  }
  return HGNN_OK;
}

int hgnn_linear_fwd(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                    const float* w, int32_t h, const float* bias, int32_t relu, float* out,
                    hgnn_stream_t stream_) {
  return hgnn_linear_fwd_add(n_seg, xs, ks, n_rows, w, h, bias, nullptr, relu, out, stream_);
}

int hgnn_linear_fwd_add(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                        const float* w, int32_t h, const float* bias, const float* add,
                        int32_t relu, float* out, hgnn_stream_t stream_) {
  return hgnn_linear_fwd_mask(n_seg, xs, ks, n_rows, w, h, bias, add, relu, out, nullptr,
                              stream_);
}

int hgnn_linear_fwd_mask(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                         const float* w, int32_t h, const float* bias, const float* add,
                         int32_t relu, float* out, uint32_t* mask, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  LinArgs a{};
  bool vec;
  if (int rc = fill_args(a, n_seg, xs, ks, nullptr, n_rows, w, h, &vec)) return rc;
  if (mask && (!relu || h % 16 != 0 || h > 128))
    return fail(HGNN_E_ARG, "linear_fwd_mask: the bit mask needs relu, h %% 16 == 0, h <= 128 (h=%d)",
                h);
  if (n_rows == 0) return HGNN_OK;
  if (out && xs_wide_ok(a, vec && reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                               reinterpret_cast<uintptr_t>(bias) % 16 == 0 &&
                               reinterpret_cast<uintptr_t>(add) % 16 == 0)) {
    a.bias = bias;
    a.add = add;
    a.out = out;
    a.relu = relu;
    a.mask_out = mask;
    if (!out_overlaps_inputs(a)) return xs_fwd_wide(a, stream);
    a.bias = nullptr; a.add = nullptr; a.out = nullptr; a.relu = 0; a.mask_out = nullptr;
  }
  if (mask && !(fwd4_ok(a, vec && reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                        reinterpret_cast<uintptr_t>(bias) % 16 == 0 &&
                        reinterpret_cast<uintptr_t>(add) % 16 == 0))) {
    // no persistent kernel for this shape: the output first, then its mask from the output
    if (int rc = hgnn_linear_fwd_add(n_seg, xs, ks, n_rows, w, h, bias, add, relu, out, stream_))
      return rc;
    hipLaunchKernelGGL(k_relu_mask, dim3((unsigned)cdiv(n_rows * 4, 256)), dim3(256), 0, stream,
                       out, n_rows, h, mask);
    return check_launch("k_relu_mask");
  }
  a.mask_out = mask;
  if (!out) return fail(HGNN_E_ARG, "linear_fwd: out is null");
  vec = vec && reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
        reinterpret_cast<uintptr_t>(bias) % 16 == 0 &&
        reinterpret_cast<uintptr_t>(add) % 16 == 0;
  if (add && !fwd4_ok(a, vec)) {
    // general shapes: the projection (no activation), then act(out + add) in one streaming pass
    if (int rc = hgnn_linear_fwd_add(n_seg, xs, ks, n_rows, w, h, bias, nullptr, 0, out,
                                     stream_))
      return rc;
    const float* ins[2] = {out, add};
    const float ws2[2] = {1.f, 1.f};
    return hgnn_hetero_epilogue(2, ins, ws2, n_rows * h, relu, out, stream_);
  }
  a.bias = bias;
  a.add = add;
  a.out = out;
  a.relu = relu;
  const unsigned gx = (unsigned)cdiv(n_rows, kRowsPerBlock);
  if (fwd4_ok(a, vec)) {
    const ChunkTab tab = chunk_table(a);
    const int64_t n_tiles = cdiv(n_rows, 16);
    const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) /
                                             ((size_t)h * (a.k_total + 8) * 4)));
    const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n_tiles, 8),
                                                                      256 * per_cu))),
        block(512);
    // the fp32-exact bf16x6 split at H = 128, K = 128 / 256 (linear_xs.hip), the default
    // (hgnn_set_k3_split(0) / HGNN_K3_X6=0: the f32-input MFMA kernel below, the one fallback)
    if (x6_enabled() && h == 128 && (a.k_total == 128 || a.k_total == 256))
      return xs_linear_fwd(a, tab, stream);
    // 128-column segment addressing where every 8 chunks are one segment (round 3: -2.5 % at
    // K = 128, -1 % at K = 256 on the cfg4 shapes; the v5 schedule measured slower with it and
    // is no longer built)
    const bool s8 = h == 128 && a.k_total >= 128 && chunks_in_segments_of_8(tab, a.k_total);
#define HGNN_FWD4A(HV, KV, AV)                                                                    \
  if (s8) hipLaunchKernelGGL((k_linear_fwd_v4<HV, KV, AV, (HV == 128 && KV >= 128)>), grid, block, \
                             0, stream, a, tab, n_tiles);                                        \
  else hipLaunchKernelGGL((k_linear_fwd_v4<HV, KV, AV, false>), grid, block, 0, stream, a, tab,  \
                          n_tiles);
#define HGNN_FWD4(HV, KV) \
  if (add) { HGNN_FWD4A(HV, KV, true) } else { HGNN_FWD4A(HV, KV, false) }
    switch (h * 1000 + a.k_total) {
      case 64064: HGNN_FWD4(64, 64); break;
      case 64128: HGNN_FWD4(64, 128); break;
      case 64256: HGNN_FWD4(64, 256); break;
      case 128064: HGNN_FWD4(128, 64); break;
      case 128128: HGNN_FWD4(128, 128); break;
      default: HGNN_FWD4(128, 256); break;
    }
#undef HGNN_FWD4
#undef HGNN_FWD4A
    return check_launch("k_linear_fwd_v4");
  }
  // v2 (W in LDS, A prefetched): 279 vs 321 us at N=1M, K=128, h=64 — the default when it fits
  bool seg16 = vec && a.k_total <= 128 && (h == 64 || h == 128);
  for (int s = 0; s < n_seg; ++s) seg16 = seg16 && ks[s] % 16 == 0;
  if (seg16) {
    const size_t lds = (size_t)h * (a.k_total + 4) * 4;
    const int kc = a.k_total / 16;
#define HGNN_FWD2(NTV, KCV) \
  hipLaunchKernelGGL((k_linear_fwd_v2<NTV, KCV>), dim3(gx), dim3(256), lds, stream, a)
    if (h == 64) {
      if (kc == 8) HGNN_FWD2(4, 8); else if (kc == 4) HGNN_FWD2(4, 4);
      else if (kc == 6) HGNN_FWD2(4, 6); else if (kc == 2) HGNN_FWD2(4, 2);
      else goto v1;
    } else {
      if (kc == 8) HGNN_FWD2(8, 8); else if (kc == 4) HGNN_FWD2(8, 4);
      else goto v1;
    }
#undef HGNN_FWD2
    return check_launch("k_linear_fwd_v2");
  }
v1:
  // few row blocks (a sampled block's 2k-32k destination rows at K = 384): 32-column tiles give
  // 4x the workgroups (measured 47 us for 2048 rows on 16 workgroups of 128 columns)
  if ((int64_t)gx * cdiv(h, 128) < 1024) {
    const dim3 grid(gx, (unsigned)cdiv(h, 32));
    if (vec) hipLaunchKernelGGL((k_linear_fwd<2, true>), grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((k_linear_fwd<2, false>), grid, dim3(256), 0, stream, a);
  } else if (h <= 64) {
    const dim3 grid(gx, 1);
    if (vec) hipLaunchKernelGGL((k_linear_fwd<4, true>), grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((k_linear_fwd<4, false>), grid, dim3(256), 0, stream, a);
  } else {
    const dim3 grid(gx, (unsigned)cdiv(h, 128));
    if (vec) hipLaunchKernelGGL((k_linear_fwd<8, true>), grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((k_linear_fwd<8, false>), grid, dim3(256), 0, stream, a);
  }
  return check_launch("k_linear_fwd");
}

static void wgrad_grid(int64_t n_rows, int32_t k_total, int32_t h, int64_t* gx, int64_t* rpb) {
  const int64_t gy = cdiv(k_total + 1, WG_K), gz = cdiv(h, WG_J);
  const int64_t tiles = cdiv(n_rows, WG_ROWS);
  int64_t want = std::max<int64_t>(1, 1024 / (gy * gz));
  const int64_t cap = std::max<int64_t>(1, (int64_t(64) << 20) / ((int64_t)h * (k_total + 1) * 4));
  want = std::min(want, cap);
  want = std::max<int64_t>(1, std::min(want, tiles));
  *rpb = cdiv(tiles, want) * WG_ROWS;
  *gx = std::max<int64_t>(1, cdiv(n_rows, *rpb));
}

size_t hgnn_linear_bwd_ws_bytes(int64_t n_rows, int32_t k_total, int32_t h) {
  int64_t gx, rpb;
  wgrad_grid(n_rows < 1 ? 1 : n_rows, k_total, h, &gx, &rpb);
  gx = std::max<int64_t>(gx, fast_grid(cdiv(n_rows < 1 ? 1 : n_rows, FT)));
  gx = std::max<int64_t>(gx, 512);   // persistent v4/v5 backward: at most 512 blocks
  return align_up((size_t)gx * h * (k_total + 1) * 4, 256) + 256;
}

int hgnn_linear_bwd(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                    const float* w, int32_t h, const float* dout, const float* out,
                    float* const* dxs, float* dw, float* db, void* ws, size_t ws_bytes,
                    hgnn_stream_t stream_) {
  return hgnn_linear_bwd_dz(n_seg, xs, ks, n_rows, w, h, dout, out, dxs, dw, db, nullptr, ws,
                            ws_bytes, stream_);
}

int hgnn_linear_bwd_dz(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                       const float* w, int32_t h, const float* dout, const float* out,
                       float* const* dxs, float* dw, float* db, float* dz_out, void* ws,
                       size_t ws_bytes, hgnn_stream_t stream_) {
  return hgnn_linear_bwd_mask(n_seg, xs, ks, n_rows, w, h, dout, out, nullptr, dxs, dw, db,
                              dz_out, ws, ws_bytes, stream_);
}

int hgnn_linear_bwd_mask(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                         const float* w, int32_t h, const float* dout, const float* out,
                         const uint32_t* mask, float* const* dxs, float* dw, float* db,
                         float* dz_out, void* ws, size_t ws_bytes, hgnn_stream_t stream_) {
  return hgnn_linear_bwd_ex(n_seg, xs, ks, n_rows, w, h, dout, out, mask, dxs, 0u, dw, db, dz_out,
                            ws, ws_bytes, stream_);
}

int hgnn_linear_bwd_ex(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                       const float* w, int32_t h, const float* dout, const float* out,
                       const uint32_t* mask, float* const* dxs, uint32_t dx_accumulate,
                       float* dw, float* db, float* dz_out, void* ws, size_t ws_bytes,
                       hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  LinArgs a{};
  bool vec;
  if (int rc = fill_args(a, n_seg, xs, ks, dxs, n_rows, w, h, &vec)) return rc;
  if (dx_accumulate >> n_seg) return fail(HGNN_E_ARG, "linear_bwd: accumulate bits beyond n_seg");
  a.dx_acc = dx_accumulate;
  if (!dout && n_rows > 0) return fail(HGNN_E_ARG, "linear_bwd: dout is null");
  if (mask && (!out || h % 16 != 0 || h > 128))
    return fail(HGNN_E_ARG, "linear_bwd_mask: the bit mask needs `out` too, h %% 16 == 0, h <= 128");
  a.dout = dout;
  a.out_act = out;
  // the persistent kernels read the bits; the others (and the streaming dz pass) read `out`
  a.mask_in = mask;
  vec = vec && reinterpret_cast<uintptr_t>(dout) % 16 == 0 &&
        (!out || reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
        reinterpret_cast<uintptr_t>(dz_out) % 16 == 0;
  for (int s = 0; s < n_seg; ++s)
    vec = vec && (!a.seg[s].dx || reinterpret_cast<uintptr_t>(a.seg[s].dx) % 16 == 0);
  if (n_rows == 0) {  // no rows: weight grads are zero
    if (dw) (void)hipMemsetAsync(dw, 0, (size_t)h * a.k_total * 4, stream);
    if (db) (void)hipMemsetAsync(db, 0, (size_t)h * 4, stream);
    return check_launch("linear_bwd(n=0)");
  }
  bool any_dx = false;
  for (int s = 0; s < n_seg; ++s) any_dx |= a.seg[s].dx != nullptr;
  if (dz_out && !(fwd4_ok(a, vec) && any_dx)) {
    // dz written by a streaming pass, then the backward from it with no mask left to apply
    const float one = 1.f;
    if (int rc = hgnn_hetero_epilogue_bwd(1, &one, n_rows * h, out ? 1 : 0, out, dout, &dz_out,
                                          stream_))
      return rc;
    return hgnn_linear_bwd_ex(n_seg, xs, ks, n_rows, w, h, dz_out, nullptr, nullptr, dxs,
                              dx_accumulate, dw, db, nullptr, ws, ws_bytes, stream_);
  }
  a.dz_out = dz_out;   // (null on the wide split path: dz_out went through the streaming pass)
  if (xs_wide_ok(a, vec) && (ws || !(dw || db)))
    return xs_bwd_wide(a, dw, db, ws, ws_bytes, stream);
  if (fwd4_ok(a, vec)) {
    // fused two-role backward when W^T and two dz / X tiles fit the LDS; otherwise persistent
    // dgrad + wgrad-only (T = 32 tiles for K = 256)
    const ChunkTab tab = chunk_table(a);
    const int K = a.k_total;
    // H = K = 128: persistent dgrad v5 + wgrad v5 (T = 16) beat the fused two-role kernel
    // (6.21 vs 8.29 ms at N = 9M); H = 64, K = 128: the fused kernel wins (3.18 vs 3.94 ms)
    const bool split = h == 128 && K == 128;
    const bool fused = !split && any_dx && (dw || db) && K <= 128 &&
                       v4_bwd_lds(h, K, true) <= 160 * 1024;
    if (x6_enabled() && h == 128 && (K == 128 || K == 256)) {
      // the split-once kernels (linear_xs.hip): dz split once for the dgrad and the wgrad
      const bool wg = dw || db;
      a.slab = nullptr;
      if (wg) {
        const size_t need = (size_t)xs_bwd_grid(n_rows) * h * (K + 1) * 4;
        if (!ws || ws_bytes < need) return fail(HGNN_E_WS, "linear_bwd: workspace too small");
        a.slab = static_cast<float*>(ws);
      }
      int G = 0;
      if (any_dx || wg) {
        if (int rc = xs_linear_bwd(a, tab, any_dx, &G, stream)) return rc;
      }
      if (!wg) return HGNN_OK;
      const int64_t total = (int64_t)h * (K + 1);
      hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)cdiv(total, 64)), dim3(1024), 0, stream,
                         a.slab, (int64_t)G, h, K + 1, dw, db, K);
      return check_launch("k_wgrad_reduce");
    }
    if (any_dx && !fused) {
      const int64_t n16 = cdiv(n_rows, 16);
      const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n16, 8), 256))),
          block(512);
      const size_t lds = dgrad4_lds(h, K);
      {
      // v5 at H = 128 (K = 256: 5.06 vs 5.70 ms; K = 128: 3.22 vs 3.25 ms at N = 9M), v4 at H = 64
#define HGNN_DG4(HV, KV)                                                                        \
  if constexpr (HV == 128)                                                                      \
    hipLaunchKernelGGL((k_linear_dgrad_v5<HV, KV>), grid, block, lds, stream, a, tab, n16);     \
  else                                                                                          \
    hipLaunchKernelGGL((k_linear_dgrad_v4<HV, KV>), grid, block, lds, stream, a, tab, n16);
      switch (h * 1000 + K) {
        case 64064: HGNN_DG4(64, 64); break;
        case 64128: HGNN_DG4(64, 128); break;
        case 64256: HGNN_DG4(64, 256); break;
        case 128064: HGNN_DG4(128, 64); break;
        case 128128: HGNN_DG4(128, 128); break;
        default: HGNN_DG4(128, 256); break;
      }
#undef HGNN_DG4
      if (int rc = check_launch("k_linear_dgrad_v4")) return rc;
      }
    }
    if (!(dw || db)) return HGNN_OK;
    if (!ws) return fail(HGNN_E_WS, "linear_bwd: weight gradients need the workspace");
    if (a.dz_out && !fused) {   // the dgrad kernel wrote the masked dz: wgrad streams it alone
      a.dout = a.dz_out;
      a.out_act = nullptr;
      a.mask_in = nullptr;
      a.dz_out = nullptr;
    }
    // wgrad v5 (every wave on MFMAs), 16-row tiles: H = K = 128 2.86 vs 4.73 ms (v4) at N = 9M;
    // v4 kept elsewhere (K = 256: v5 6.44 / 9.51 ms at T = 16 / 32 vs 5.65; H = 64 needs T >= 32,
    // which measured slower than v4: 2.44 vs 1.94 ms)
    constexpr int wg_t = 16;
    if (!fused && h == 128 && K == 128) {
      const int64_t n_tiles = cdiv(n_rows, wg_t);
      const size_t lds = wgrad5_lds(h, K, wg_t);
      const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / lds));
      const int G = (int)std::min<int64_t>(n_tiles, 256 * per_cu);
      const size_t need = (size_t)G * h * (K + 1) * 4;
      if (ws_bytes < need) return fail(HGNN_E_WS, "linear_bwd: workspace too small");
      a.slab = static_cast<float*>(ws);
      const dim3 grid(G), block(512);
      hipLaunchKernelGGL((k_linear_wgrad_v5<128, 128, wg_t>), grid, block, lds, stream, a, tab,
                         n_tiles);
      if (int rc = check_launch("k_linear_wgrad_v5")) return rc;
      const int64_t total = (int64_t)h * (K + 1);
      hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)cdiv(total, 64)), dim3(1024), 0, stream,
                         a.slab, (int64_t)G, h, K + 1, dw, db, K);
      return check_launch("k_wgrad_reduce");
    }
    const int T = v4_bwd_lds(h, K, fused, 64) <= 160 * 1024 ? 64 : 32;
    const int64_t n_tiles = cdiv(n_rows, T);
    const int G = (int)std::min<int64_t>(n_tiles, 256);
    const size_t lds = v4_bwd_lds(h, K, fused, T);
    const size_t need = (size_t)G * h * (K + 1) * 4;
    if (ws_bytes < need) return fail(HGNN_E_WS, "linear_bwd: workspace too small");
    a.slab = static_cast<float*>(ws);
    const dim3 grid(G), block(512);
#define HGNN_BWD4(HV, KV, DXV, TV) \
  hipLaunchKernelGGL((k_linear_bwd_v4<HV, KV, DXV, TV>), grid, block, lds, stream, a, tab, n_tiles)
    if (fused) {
      switch (h * 1000 + K) {
        case 64064: HGNN_BWD4(64, 64, true, 64); break;
        case 64128: HGNN_BWD4(64, 128, true, 64); break;
        default: HGNN_BWD4(128, 64, true, 64); break;
      }
    } else {
      switch (h * 1000 + K) {
        case 64064: HGNN_BWD4(64, 64, false, 64); break;
        case 64128: HGNN_BWD4(64, 128, false, 64); break;
        case 64256: HGNN_BWD4(64, 256, false, 32); break;
        case 128064: HGNN_BWD4(128, 64, false, 64); break;
        case 128128: HGNN_BWD4(128, 128, false, 64); break;
        default: HGNN_BWD4(128, 256, false, 32); break;
      }
    }
#undef HGNN_BWD4
    if (int rc = check_launch("k_linear_bwd_v4")) return rc;
    const int64_t total = (int64_t)h * (K + 1);
    hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)cdiv(total, 64)), dim3(1024), 0, stream,
                       a.slab, (int64_t)G, h, K + 1, dw, db, K);
    return check_launch("k_wgrad_reduce");
  }
  if (fast_path_ok(a, vec) && (dw || db) && ws) {
    const int64_t n_tiles = cdiv(n_rows, FT);
    const int G = fast_grid(n_tiles);
    const size_t need = (size_t)G * h * (a.k_total + 1) * 4;
    if (ws_bytes < need) return fail(HGNN_E_WS, "linear_bwd: workspace too small");
    a.slab = static_cast<float*>(ws);
    const size_t lds = ((size_t)a.k_total * (h + 4) + (size_t)FT * (h + 16) +
                        (size_t)FT * (a.k_total + 16)) * 4;
    const dim3 grid(G), block(256);
#define HGNN_BWD_LDS(NTV)                                                                      \
  if (any_dx) hipLaunchKernelGGL((k_linear_bwd_lds<NTV, true>), grid, block, lds, stream, a,   \
                                 n_tiles);                                                     \
  else hipLaunchKernelGGL((k_linear_bwd_lds<NTV, false>), grid, block, lds, stream, a, n_tiles);
    switch (h / 16) {
      case 1: HGNN_BWD_LDS(1) break;
      case 2: HGNN_BWD_LDS(2) break;
      case 4: HGNN_BWD_LDS(4) break;
      case 8: HGNN_BWD_LDS(8) break;
      default: return fail(HGNN_E_UNSUPPORTED, "linear_bwd fast path: h=%d", h);
    }
#undef HGNN_BWD_LDS
    if (int rc = check_launch("k_linear_bwd_lds")) return rc;
    const int64_t total = (int64_t)h * (a.k_total + 1);
    hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)cdiv(total, 64)), dim3(1024), 0, stream,
                       a.slab, (int64_t)G, h, a.k_total + 1, dw, db, a.k_total);
    return check_launch("k_wgrad_reduce");
  }
  if (any_dx) {
    const int64_t gxd = cdiv(n_rows, kRowsPerBlock);
    if (gxd * cdiv(a.k_total, 128) < 1024) {   // few row blocks: 32-column tiles (see forward)
      const dim3 grid((unsigned)gxd, (unsigned)cdiv(a.k_total, 32));
      if (vec) hipLaunchKernelGGL((k_linear_dgrad<2, true>), grid, dim3(256), 0, stream, a);
      else hipLaunchKernelGGL((k_linear_dgrad<2, false>), grid, dim3(256), 0, stream, a);
    } else {
      const dim3 grid((unsigned)gxd, (unsigned)cdiv(a.k_total, 128));
      if (vec) hipLaunchKernelGGL((k_linear_dgrad<8, true>), grid, dim3(256), 0, stream, a);
      else hipLaunchKernelGGL((k_linear_dgrad<8, false>), grid, dim3(256), 0, stream, a);
    }
    if (int rc = check_launch("k_linear_dgrad")) return rc;
  }
  if (dw || db) {
    int64_t gx, rpb;
    wgrad_grid(n_rows, a.k_total, h, &gx, &rpb);
    const size_t need = (size_t)gx * h * (a.k_total + 1) * 4;
    if (!ws || ws_bytes < need) return fail(HGNN_E_WS, "linear_bwd: workspace too small");
    a.slab = static_cast<float*>(ws);
    a.rows_per_block = rpb;
    const dim3 grid((unsigned)gx, (unsigned)cdiv(a.k_total + 1, WG_K), (unsigned)cdiv(h, WG_J));
    if (vec) hipLaunchKernelGGL(k_linear_wgrad<true>, grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL(k_linear_wgrad<false>, grid, dim3(256), 0, stream, a);
    if (int rc = check_launch("k_linear_wgrad")) return rc;
    const int64_t total = (int64_t)h * (a.k_total + 1);
    hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)cdiv(total, 64)), dim3(1024), 0, stream,
                       a.slab, gx, h, a.k_total + 1, dw, db, a.k_total);
    if (int rc = check_launch("k_wgrad_reduce")) return rc;
  }
  return HGNN_OK;
}

int hgnn_set_k3_split(int32_t on) {
  const int prev = x6_enabled() ? 1 : 0;
  if (on >= 0) g_k3_x6 = on ? 1 : 0;
  return prev;
}

// ---- single-input forms (the PyG Linear calls one at a time; SURVEY §8b names) ----------------
// lin(x) = x @ w^T (+ bias): PyG Linear inside SAGEConv (lin_l with bias, lin_r without).
int hgnn_linear_fwd_f32(const float* x, int64_t n_rows, int32_t k, const float* w, int32_t h,
                        const float* bias, float* out, hgnn_stream_t stream) {
  return hgnn_linear_fwd(1, &x, &k, n_rows, w, h, bias, 0, out, stream);
}

// dx = dy @ w (autograd of lin).  The dx-only backward never reads x, so dx stands in for it.
int hgnn_linear_dgrad_f32(const float* dy, int64_t n_rows, int32_t h, const float* w, int32_t k,
                          float* dx, hgnn_stream_t stream) {
  if (n_rows > 0 && !dx) return fail(HGNN_E_ARG, "linear_dgrad: dx is null");
  const float* x = dx;
  return hgnn_linear_bwd(1, &x, &k, n_rows, w, h, dy, nullptr, &dx, nullptr, nullptr, nullptr, 0,
                         stream);
}

// dw = dy^T @ x, db = colsum(dy) (db may be NULL).  ws: hgnn_linear_bwd_ws_bytes(n_rows, k, h).
// The weight-only backward never reads w (every W load sits behind the dx template flag), so dw
// stands in for it.
int hgnn_linear_wgrad_f32(const float* x, const float* dy, int64_t n_rows, int32_t k, int32_t h,
                          float* dw, float* db, void* ws, size_t ws_bytes, hgnn_stream_t stream) {
  if (!dw) return fail(HGNN_E_ARG, "linear_wgrad: dw is null");
  return hgnn_linear_bwd(1, &x, &k, n_rows, dw, h, dy, nullptr, nullptr, dw, db, ws, ws_bytes,
                         stream);
}

}  // extern "C"
