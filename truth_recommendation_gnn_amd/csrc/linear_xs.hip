// K3 on the fp32-exact bf16x6 split, split once per element (round 4).  Replaces SAGEConv's
// lin_l / lin_r addmm plus WeightedRGCN's weighted sum, bias and ReLU (train_gnn.py:158-160,
// 187-198) and their autograd at H = 128, K = 128 / 256: the cfg3 / cfg4 projections.
//
// The round-3 split kernels (linear.hip, k_linear_*_x6) loaded X in the MFMA fragment layout —
// 64 B of a row per lane group per load instruction — and every wave split the values it loaded
// (at K = 256 twice, once per column half).  They ran at 0.37-0.43 of the HBM roof, bound by
// neither HBM nor MFMA.  Here a block stages R-row tiles with whole-row coalesced float4 loads
// (a wave reads 1 KiB of contiguous row per instruction), splits each element ONCE into three
// bf16 piece planes in LDS, and all 8 waves take their MFMA operands from those planes:
//   * forward: wave w owns output columns 16 w .. 16 w + 15; its W pieces live in VGPRs for the
//     whole launch, the tile's X pieces come from LDS (ds_read_b128 row fragments);
//   * backward: the masked dz tile is split once and serves BOTH the dgrad (ds_read_b128 row
//     fragments, W^T pieces in VGPRs) and the wgrad (ds_read_b64_tr_b16 transposed fragments,
//     with the X tile's planes), so dz and X are each read from HBM once per launch.
// Double-buffered planes, one barrier per tile; the next tile's loads are issued at the top of
// an iteration and split into the other buffer after its MFMA sweep.
//
// LDS piece planes are [row][K + 16 halfwords]: rows 32 B apart mod 256 B, so the b128 row
// fragment reads (lanes (i, g): row i, 16 B at 8 g) and the b64 transposed reads (see tr8) are
// conflict-free, and each 16-lane group of the staging ds_write_b64 writes 128 contiguous bytes.
#include "linear_common.h"

#include <algorithm>
#include <stdlib.h>
#include <type_traits>

#ifndef HGNN_XS_LDSPF
#define HGNN_XS_LDSPF 2
#endif
#ifndef HGNN_XS_LDSPF_DXWG
#define HGNN_XS_LDSPF_DXWG 1
#endif

namespace hgnn {

namespace {

constexpr int kH = 128;     // output width
constexpr int kThr = 512;   // 8 waves

typedef short v4s __attribute__((ext_vector_type(4)));

// row clamp (a mixed-type min<int64_t>(int64, int32) compiled to f64 converts and v_min_f64)
__device__ __forceinline__ uint32_t clamp_row(int64_t row, int32_t last) {
  return min((uint32_t)row, (uint32_t)last);   // row < 2^32: n < 2^31 and at most 2 G R past it
}
typedef __attribute__((address_space(3))) v4s lds_v4s;

typedef uint32_t xs_u32x2 __attribute__((ext_vector_type(2)));

// One [R x K] fp32 tile of the concatenated input, staged by all 512 threads: float4 j of thread
// t is f = t + 512 j, row f / (K / 4), column 4 (f % (K / 4)) — a thread's column (and therefore
// its 16-column chunk of the ChunkTab) is fixed, its rows step by 512 / (K / 4).  Row indices
// are 32-bit (the host checks n < 2^31): one v_mad_u64_u32 per row address.
template <int K, int R, int THR = kThr>
struct XStage {
  static constexpr int NL = R * K / 4 / THR;
  static constexpr int RSTEP = THR / (K / 4);
  struct Regs {
    float4 v[NL];
  };
  const float* base;
  uint32_t ld;
  int row0, col;
  __device__ __forceinline__ void init(const ChunkTab& tab) {
    col = 4 * ((int)threadIdx.x % (K / 4));
    row0 = (int)threadIdx.x / (K / 4);
    const int c = col >> 4;
    base = tab.x[c] + tab.col[c] + (col & 15);
    ld = (uint32_t)tab.ld[c];
  }
  // rows past the end are clamped to the last row (loaded, never stored).  (Measured and not
  // kept: a uniform in-range test per tile taking one v_mad_u64_u32 and 64-bit adds for the row
  // addresses — fewer VALU, but 3.42 -> 3.46 ms at K = 256 forward, 3.55 -> 3.64 backward.)
  __device__ __forceinline__ void issue_one(Regs& x, int64_t r0, int32_t last, int j) const {
    const uint32_t row = clamp_row(r0 + row0 + j * RSTEP, last);
    x.v[j] = *reinterpret_cast<const float4*>(base + (uint64_t)row * ld);
  }
  __device__ __forceinline__ void issue(Regs& x, int64_t r0, int32_t last) const {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const uint32_t row = clamp_row(r0 + row0 + j * RSTEP, last);
      x.v[j] = *reinterpret_cast<const float4*>(base + (uint64_t)row * ld);
    }
  }
  // split into the three planes (plane stride PS halfwords, row stride LDP).  Rows past the end
  // are clamped copies of the last row: a forward row only reaches its own (unstored) output,
  // and the backward pairs them with zeroed dz rows
  template <int LDP, int PS>
  __device__ __forceinline__ void put(const Regs& x, unsigned short* pl) const {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      bf16x4_t p1, p2, p3;
      x6_split4(x.v[j], p1, p2, p3);
      unsigned short* d = pl + (row0 + j * RSTEP) * LDP + col;
      *reinterpret_cast<bf16x4_t*>(d) = p1;
      *reinterpret_cast<bf16x4_t*>(d + PS) = p2;
      *reinterpret_cast<bf16x4_t*>(d + 2 * PS) = p3;
    }
  }
};

// b128 row fragment of a plane: lane (i, g) reads row r0 + i, halfwords c0 + 8 g .. + 7
template <int LDP>
__device__ __forceinline__ bf16x8_t row8(const unsigned short* pl, int r0, int c0, int i, int g) {
  return *reinterpret_cast<const bf16x8_t*>(pl + (r0 + i) * LDP + c0 + 8 * g);
}

// Transposed fragment of a [32 rows][LDP] plane for an MFMA operand whose reduction index runs
// over the tile's rows: lane (i, g) receives column c0 + i at the rows of its k slots.  The
// reduction index k = 8 g + kk maps to tile row 4 g + kk (kk < 4) and 16 + 4 g + kk - 4
// (kk >= 4) — any bijection does, the same for both operands — so each 32-lane half of a
// ds_read_b64_tr_b16 reads 8 consecutive rows (32 B each at 32 B apart mod 256): conflict-free.
// Lane 4 q + p of a 16-lane group addresses row q of its 4-row block, columns 4 p .. 4 p + 3.
template <int LDP>
__device__ __forceinline__ bf16x8_t tr8(const unsigned short* pl, int c0, int lane) {
  const int g = lane >> 4, m = lane & 15;
  const unsigned short* p = pl + (4 * g + (m >> 2)) * LDP + c0 + 4 * (m & 3);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p + 16 * LDP));
  bf16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// ---------------------------------------------------------------- forward
// out[n, 0:128] = act(sum_s X_s W_s^T + b (+ add)), tiles of R rows (R * K * 4 = 32 KB of X).
// MFMA: A = W pieces (rows = output columns 16 w + i), B = X^T from the planes, so lane (i, g)
// ends with columns 16 w + 4 g .. +3 of tile row 16 r + i: float4 stores; the ReLU mask words
// (bit 4 c + e of word row * 4 + g) collect each wave's nibble through an LDS OR.
// Per tile: [MFMA sweep, with the iteration's memory instructions one or two per sweep step]
// [epilogue into registers] [split of the next tile into the other buffer] [barrier].
// Memory order matters because vmcnt is one in-order counter: a wait on an operation also waits
// for everything issued before it.  The outputs are stored during the NEXT iteration's sweep, and
// their registers are held until after it: the compiler waits for a store to read its data before
// it lets anything overwrite those registers, and with the stores issued last (before the
// barrier) that wait landed at the loop head and drained the prefetch with them.  The prefetch is
// unconditional (past the last tile the rows clamp and the split goes to an unread buffer): a
// conditional issue made the waitcnt pass assume loads in flight at the loop head and wait for
// everything there.  For the same reason the stores inside the loop are unconditional: a tile
// before a block's last is full (only tile n_tiles - 1 is partial, and it is some block's last),
// and a store under a branch counts as maybe-not-issued, so the epilogue's wait for the added rows
// had waited for every store as well (round 6).
// The memory instructions spread over the sweep (round 5): in-kernel stamps (scripts/k3_stamps.py)
// had shown all 8 waves queueing ~48 KB of requests on the CU's memory pipe right after the
// barrier, ~600 cycles each, while the matrix pipe sat idle.  A/B at the cfg4 shapes: K = 128 +
// add 2.589 -> 2.512 ms, K = 128 (preprojection, 1M rows) 0.219 -> 0.198, K = 256 unchanged.
// Measured and not kept: a prefetch two tiles deep; the split interleaved into
// the sweep; the burst issued at a later sweep step; the split level by level for ILP; the bias as
// the accumulator's initial value; the output tile staged in LDS and stored as whole rows.
// (bid, G): the block's index and the block count of its job — blockIdx.x / gridDim.x in a
// launch of its own, the job's range of a two-job launch (k_lin_fwd_xs2)
template <int K, bool ADD>
__device__ __forceinline__ void lin_fwd_xs_body(const LinArgs& a, const ChunkTab& tab,
                                                int64_t n_tiles, uint32_t bid, uint32_t G_) {
  const int64_t G = G_;
  constexpr int R = K == 256 ? 32 : 64, KS = K / 32, RT = R / 16, LDP = K + 16, PS = R * LDP;
  constexpr int NA = ADD ? RT : 0, NX = XStage<K, R>::NL;
  __shared__ __attribute__((aligned(16))) unsigned short pl[2][3 * PS];
  __shared__ uint32_t mk[2][R * 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int32_t last = (int32_t)(a.n - 1);
  // W pieces of this wave's 16 output columns, for the whole launch
  bf16x8_t wa[KS][3];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const float4* p = reinterpret_cast<const float4*>(a.w + (int64_t)(16 * w + i) * a.ldw + 32 * s +
                                                      8 * g);
    x6_split8(p[0], p[1], wa[s][0], wa[s][1], wa[s][2]);
  }
  const float4 bb = a.bias ? *reinterpret_cast<const float4*>(a.bias + 16 * w + 4 * g)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
  const bool mask_out = a.mask_out != nullptr;
  for (int e = threadIdx.x; e < 2 * R * 4; e += kThr) (&mk[0][0])[e] = 0u;
  XStage<K, R> xs;
  xs.init(tab);
  typename XStage<K, R>::Regs xr;
  float4 ad[ADD ? RT : 1];
  float4 po[RT];   // the previous tile's output rows
#pragma unroll
  for (int r = 0; r < RT; ++r) po[r] = make_float4(0.f, 0.f, 0.f, 0.f);
  // FULL: a tile before the block's last (every row < n), stored without a row test
  auto store_one = [&](int64_t tp, int r, auto full_c) {
    const int64_t row = tp * R + 16 * r + i;
    if (decltype(full_c)::value || row < a.n)
      *reinterpret_cast<float4*>(a.out + row * kH + 16 * w + 4 * g) = po[r];
  };
  auto mask_one = [&](int64_t tp, int bp, auto full_c) {
    if (mask_out && threadIdx.x < R * 4) {   // its mask words are complete (last barrier)
      const int64_t row = tp * R + (threadIdx.x >> 2);
      if (decltype(full_c)::value || row < a.n)
        a.mask_out[tp * R * 4 + threadIdx.x] = mk[bp][threadIdx.x];
      mk[bp][threadIdx.x] = 0u;
    }
  };
  int64_t t = bid;   // the job's grid never exceeds its n_tiles
  xs.issue(xr, t * R, last);
  xs.template put<LDP, PS>(xr, pl[0]);
  // Staggered halves (HGNN_XS_STAGGER): the two waves sharing a SIMD (w and w + 4) run the same
  // program in lockstep, so both sweep (matrix pipe busy, VALU idle) and then both split (VALU
  // busy, matrix pipe idle).  Waves 4-7 instead split the next tile FIRST — from loads issued an
  // iteration earlier — and sweep after, so each SIMD pairs one wave's MFMAs with its partner's
  // split.  Both orders write the other buffer and read this one between the same two barriers.
  // A/B at the cfg4 9M-row shapes: K = 256 3.75 -> 3.59 ms, K = 128 + add 2.74 -> 2.67 ms, the
  // backward unchanged (within noise); `s_setprio 1` for waves 4-7 on top was slower.  Also
  // measured and not kept: 4 waves of 512 registers, each with 32 output columns (half the LDS
  // reads per MFMA) and the next tile's split interleaved into its own sweep by scheduling group
  // barriers — correct, but 3.39 -> 3.78 ms at K = 256, 2.59 -> 2.84 ms at K = 128 + add; and
  // specialised waves (12 per block: 8 MFMA waves as here, 4 that only load and split, one per
  // SIMD) — 3.41 -> 3.37 ms and 2.61 -> 2.50 ms, at the 168-register limit of three waves per
  // SIMD (spills at K = 256 + add): too little for a second forward kernel.  Larger tiles (48
  // rows at K = 256, 80 at K = 128: fewer barriers and epilogue phases per MFMA) measured the
  // same (3.52 / 3.49 ms, 2.68 / 2.69 ms).
  auto loop = [&](auto late_c) {
    constexpr bool LATE = decltype(late_c)::value;
    if constexpr (LATE) xs.issue(xr, (t + G) * R, last);
    __syncthreads();
    int it = 0;
    // the first iteration peeled (FIRST: no previous tile to store), so the stores of every
    // other iteration are unconditional and the compiler's waits count them
    auto iter = [&](auto first_c) {
      constexpr bool FIRST = decltype(first_c)::value;
      const int b = it & 1;
      if constexpr (LATE) xs.template put<LDP, PS>(xr, pl[b ^ 1]);
      // the iteration's memory instructions, piece k at sweep step k * NQ / NP: the previous
      // tile's mask words, this tile's added rows, the prefetch, the previous tile's stores
      // (youngest: the waits for the added rows and the prefetch leave them in flight)
      auto vmem_step = [&](int q) {
        constexpr int NP = 1 + NA + NX + RT, NQ = RT * KS;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          if (k * NQ / NP != q) continue;
          if (k == 0) {
            if constexpr (!FIRST) mask_one(t - G, b ^ 1, std::true_type{});
          } else if (k < 1 + NA) {
            if constexpr (ADD) {
              const uint32_t row = clamp_row(t * R + 16 * (k - 1) + i, last);
              ad[k - 1] =
                  *reinterpret_cast<const float4*>(a.add + (uint64_t)row * kH + 16 * w + 4 * g);
            }
          } else if (k < 1 + NA + NX) {
            xs.issue_one(xr, (t + (LATE ? 2 : 1) * G) * R, last, k - 1 - NA);
          } else {
            if constexpr (!FIRST) store_one(t - G, k - 1 - NA - NX, std::true_type{});
          }
        }
      };
      const unsigned short* p = pl[b];
      f32x4 hi[RT], lo[RT];
      // software-pipelined sweep: step q = (r, s) reads its three fragments LDSPF steps ahead,
      // pinned as [3 ds_read (step q + LDSPF)] [6 MFMA (step q)] by scheduling barriers (the
      // compiler otherwise issues each step's reads right before its MFMAs and waits on them)
      {
        constexpr int NQ = RT * KS, PF = HGNN_XS_LDSPF;
        bf16x8_t fr[PF + 1][3];
        auto ld = [&](int q, bf16x8_t (&f)[3]) {
          const int r = q / KS, s2 = q % KS;
          f[0] = row8<LDP>(p, 16 * r, 32 * s2, i, g);
          f[1] = row8<LDP>(p + PS, 16 * r, 32 * s2, i, g);
          f[2] = row8<LDP>(p + 2 * PS, 16 * r, 32 * s2, i, g);
        };
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          hi[r] = f32x4{0.f, 0.f, 0.f, 0.f};
          lo[r] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int q = 0; q < PF; ++q) ld(q, fr[q]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          vmem_step(q);
          if (q + PF < NQ) ld(q + PF, fr[(q + PF) % (PF + 1)]);
          __builtin_amdgcn_sched_barrier(0);
          x6_mma(wa[q % KS], fr[q % (PF + 1)][0], fr[q % (PF + 1)][1], fr[q % (PF + 1)][2],
                 hi[q / KS], lo[q / KS]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // the stored rows' registers are reserved until here (see above)
#pragma unroll
      for (int r = 0; r < RT; ++r)
        asm volatile("" ::"v"(po[r].x), "v"(po[r].y), "v"(po[r].z), "v"(po[r].w));
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        float4 v = make_float4(x6_out(hi[r][0], lo[r][0]) + bb.x, x6_out(hi[r][1], lo[r][1]) + bb.y,
                               x6_out(hi[r][2], lo[r][2]) + bb.z, x6_out(hi[r][3], lo[r][3]) + bb.w);
        if constexpr (ADD) {
          v.x += ad[r].x; v.y += ad[r].y; v.z += ad[r].z; v.w += ad[r].w;
        }
        if (a.relu) v = relu4(v);
        po[r] = v;
        if (mask_out) atomicOr(&mk[b][(16 * r + i) * 4 + g], relu_out_bits(v, 4 * w));
      }
      if constexpr (!LATE) xs.template put<LDP, PS>(xr, pl[b ^ 1]);
      __syncthreads();
    };
    if (t < n_tiles) {
      iter(std::true_type{});
      t += G;
      ++it;
    }
    for (; t < n_tiles; t += G, ++it) iter(std::false_type{});
#pragma unroll
    for (int r = 0; r < RT; ++r) store_one(t - G, r, std::false_type{});
    mask_one(t - G, (it - 1) & 1, std::false_type{});
  };
  if (w >= 4) {
    loop(std::true_type{});
  } else {
    loop(std::false_type{});
  }
}

template <int K, bool ADD>
__global__ void __launch_bounds__(kThr, 1) k_lin_fwd_xs(const LinArgs a, const ChunkTab tab,
                                                        int64_t n_tiles) {
  lin_fwd_xs_body<K, ADD>(a, tab, n_tiles, blockIdx.x, gridDim.x);
}

// Two jobs of the same shape class in one launch (two destination types' projections of a
// layer): blocks [0, g0) run job 0, the rest job 1, each a persistent grid of its own.
template <int K, bool ADD>
__global__ void __launch_bounds__(kThr, 1) k_lin_fwd_xs2(const XsPair p) {
  const int j = blockIdx.x < (uint32_t)p.g0 ? 0 : 1;
  const uint32_t g0 = (uint32_t)p.g0;
  const uint32_t bid = j ? blockIdx.x - g0 : blockIdx.x;
  const uint32_t G = j ? gridDim.x - g0 : g0;
  lin_fwd_xs_body<K, ADD>(p.a[j], p.tab[j], p.n_tiles[j], bid, G);
}

// ---------------------------------------------------------------- backward
// Per 32-row tile: dz = dout masked by the ReLU bits (or by out > 0, or none), written to dz_out
// when asked, summed for db, split into planes; X split into planes.  Then
//   DX: dX^T = W^T dz^T (wave w owns the dX column tiles w + 8 u, u < K / 128 — 16-column
//       chunks of the ChunkTab); A = W^T pieces in VGPRs, B = dz row fragments (K = 256 with
//       the wgrad too would not fit the registers: the host runs that as two launches);
//   WG: dW += dz^T X over the tile's 32 rows (one MFMA k-step): wave w owns dW columns
//       [KW w, KW w + KW), KW = K / 8, every h; A = transposed dz fragments, B = transposed X.
// The block's dW / db partials go to its slab [H][K + 1] (k_wgrad_reduce sums them in order).
template <int K, bool DX, bool WG, bool ACC>
__device__ __forceinline__ void lin_bwd_xs_body(const LinArgs& a, const ChunkTab& tab,
                                                int64_t n_tiles, uint32_t bid, uint32_t G_) {
  const int64_t G = G_;
  static_assert(!(DX && WG) || K == 128, "dgrad + wgrad in one pass: K = 128");
  constexpr int R = 32, LDZ = kH + 16, LDX = K + 16, ZS = R * LDZ, XS = R * LDX;
  constexpr int KT = K / 128;      // 16-column k tiles of dW per wave
  constexpr int HS = kH / 32;      // dgrad MFMA k-steps (reduction over h)
  __shared__ __attribute__((aligned(16))) unsigned short zp[2][3 * ZS];
  __shared__ __attribute__((aligned(16))) unsigned short xp[WG ? 2 : 1][WG ? 3 * XS : 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int32_t last32 = (int32_t)(a.n - 1);
  const bool bits = a.mask_in != nullptr;
  const bool masked = !bits && a.out_act != nullptr;
  // dgrad: W^T pieces of dX columns 16 (w + 8 u) + i, h = 32 s + 8 g .. +7
  constexpr int DT = DX ? KT : 1;
  bf16x8_t wt[DT][DX ? HS : 1][3];
  if constexpr (DX) {
#pragma unroll
    for (int u = 0; u < DT; ++u)
#pragma unroll
      for (int s = 0; s < HS; ++s) {
        float f[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          f[e] = a.w[(int64_t)(32 * s + 8 * g + e) * a.ldw + 16 * (w + 8 * u) + i];
        x6_split8(make_float4(f[0], f[1], f[2], f[3]), make_float4(f[4], f[5], f[6], f[7]),
                  wt[u][s][0], wt[u][s][1], wt[u][s][2]);
      }
  }
  // dz staging: float4 j of thread t at row (t >> 5) + 16 j, columns 4 (t & 31) .. +3
  constexpr int ZL = 2;
  const int zc = 4 * (threadIdx.x & 31), zr = threadIdx.x >> 5;
  const int msh = 4 * (zc >> 4);      // bits of column tile zc / 16 in word row * 4 + (zc / 4) % 4
  float4 zv[ZL], mv[ZL];
  uint32_t mw[ZL];
  XStage<K, R> xs;
  typename XStage<K, R>::Regs xr;
  if constexpr (WG) xs.init(tab);
  auto issue = [&](int64_t tt) {
#pragma unroll
    for (int j = 0; j < ZL; ++j) {
      const uint64_t row = clamp_row(tt * R + zr + 16 * j, last32);
      zv[j] = *reinterpret_cast<const float4*>(a.dout + row * kH + zc);
      if (bits) mw[j] = a.mask_in[row * 4 + ((zc >> 2) & 3)];
      if (masked) mv[j] = *reinterpret_cast<const float4*>(a.out_act + row * kH + zc);
    }
    if constexpr (WG) xs.issue(xr, tt * R, last32);
  };
  float4 dbacc = make_float4(0.f, 0.f, 0.f, 0.f);
  auto put = [&](int64_t tt, int b) {
#pragma unroll
    for (int j = 0; j < ZL; ++j) {
      const int64_t row = tt * R + zr + 16 * j;
      float4 z = zv[j];
      if (bits) z = mask4(z, mw[j], msh);
      if (masked) {
        const float4 m = mv[j];
        z.x = m.x > 0.f ? z.x : 0.f; z.y = m.y > 0.f ? z.y : 0.f;
        z.z = m.z > 0.f ? z.z : 0.f; z.w = m.w > 0.f ? z.w : 0.f;
      }
      if (row >= a.n) z = make_float4(0.f, 0.f, 0.f, 0.f);
      else if (a.dz_out) *reinterpret_cast<float4*>(a.dz_out + row * kH + zc) = z;
      dbacc.x += z.x; dbacc.y += z.y; dbacc.z += z.z; dbacc.w += z.w;
      bf16x4_t p1, p2, p3;
      x6_split4(z, p1, p2, p3);
      unsigned short* d = zp[b] + (zr + 16 * j) * LDZ + zc;
      *reinterpret_cast<bf16x4_t*>(d) = p1;
      *reinterpret_cast<bf16x4_t*>(d + ZS) = p2;
      *reinterpret_cast<bf16x4_t*>(d + 2 * ZS) = p3;
    }
    // X's rows past n are NOT zeroed (round 6): they are clamped copies of row n - 1 and meet
    // only the zeroed dz rows above, so their products are exact zeros — unless row n - 1 holds
    // an inf or NaN, where 0 x inf adds NaN to the columns the f32 kernels would make +-inf.
    // Saves a compare and four selects per float4 on every tile.
    if constexpr (WG) xs.template put<LDX, XS>(xr, xp[b]);
  };
  // (Measured and not kept: a uniform branch to a copy of the put without the per-row zeroing
  // on every tile but the last — within noise at the cfg4 shapes, and the K = 256 wgrad kernel
  // spills with the second copy.)
  f32x4 hw[WG ? 8 : 1][KT], lw[WG ? 8 : 1][KT];
#pragma unroll
  for (int h = 0; h < (WG ? 8 : 1); ++h)
#pragma unroll
    for (int u = 0; u < KT; ++u) hw[h][u] = lw[h][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  // dgrad: this wave's dX column tiles are chunks w + 8 u, loop-invariant
  float* dxp[DT];
  int64_t dxld[DT];
  bool acc_dx[DT];
#pragma unroll
  for (int u = 0; u < DT; ++u) {
    const int c = w + 8 * u;
    dxp[u] = DX && tab.dx[c] ? tab.dx[c] + tab.col[c] : nullptr;
    dxld[u] = DX ? tab.ld[c] : 0;
    acc_dx[u] = DX && ((tab.dx_acc >> c) & 1u);
  }
  int64_t t = bid;   // the job's grid never exceeds its n_tiles
  issue(t);
  put(t, 0);
  // staggered halves as in the forward: waves 4-7 put the next tile first, then sweep
  auto loop = [&](auto late_c) {
    constexpr bool LATE = decltype(late_c)::value;
    if constexpr (LATE) issue(t + G);
    __syncthreads();
    for (int it = 0; t < n_tiles; t += G, ++it) {
      const int b = it & 1;
      if constexpr (LATE) put(t + G, b ^ 1);
      // an accumulating dX reads what the rows hold first: issued before the prefetch, so its
      // wait leaves the prefetch in flight
      float4 dxo[DT][ACC ? R / 16 : 1];
      if constexpr (ACC) {
#pragma unroll
        for (int u = 0; u < DT; ++u) {
          if (dxp[u]) {
#pragma unroll
            for (int r = 0; r < R / 16; ++r)
              dxo[u][r] = *reinterpret_cast<const float4*>(
                  dxp[u] + (uint64_t)clamp_row(t * R + 16 * r + i, last32) * dxld[u] + 4 * g);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      issue(t + (LATE ? 2 : 1) * G);   // consumed by the next put(), unconditionally (see forward)
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of what follows
      const unsigned short* z = zp[b];
      f32x4 dh[DT][DX ? R / 16 : 1], dl[DT][DX ? R / 16 : 1];
      // the sweeps software-pipelined as in the forward: each step's fragments are read PF
      // steps ahead, pinned by scheduling barriers; the fused dgrad + wgrad kernels are at the
      // register limit: fewer fragments ahead there
      constexpr int PF = DX && WG ? (ACC ? 0 : HGNN_XS_LDSPF_DXWG) : HGNN_XS_LDSPF;
      if constexpr (DX) {
        constexpr int NQ = (R / 16) * HS;
        bf16x8_t fr[PF + 1][3];
        auto ld = [&](int q, bf16x8_t (&f)[3]) {
          const int r = q / HS, s2 = q % HS;
          f[0] = row8<LDZ>(z, 16 * r, 32 * s2, i, g);
          f[1] = row8<LDZ>(z + ZS, 16 * r, 32 * s2, i, g);
          f[2] = row8<LDZ>(z + 2 * ZS, 16 * r, 32 * s2, i, g);
        };
#pragma unroll
        for (int r = 0; r < R / 16; ++r)
#pragma unroll
          for (int u = 0; u < DT; ++u) dh[u][r] = dl[u][r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < PF; ++q) ld(q, fr[q]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          if (q + PF < NQ) ld(q + PF, fr[(q + PF) % (PF + 1)]);
          __builtin_amdgcn_sched_barrier(0);
          const bf16x8_t(&f)[3] = fr[q % (PF + 1)];
#pragma unroll
          for (int u = 0; u < DT; ++u)
            x6_mma(wt[u][q % HS], f[0], f[1], f[2], dh[u][q / HS], dl[u][q / HS]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if constexpr (WG) {
        const unsigned short* x = xp[b];
        bf16x8_t xb[KT][3];
#pragma unroll
        for (int u = 0; u < KT; ++u)
#pragma unroll
          for (int q = 0; q < 3; ++q) xb[u][q] = tr8<LDX>(x + q * XS, 16 * (KT * w + u), lane);
        bf16x8_t za[PF + 1][3];
#pragma unroll
        for (int h = 0; h < PF; ++h)
#pragma unroll
          for (int q = 0; q < 3; ++q) za[h][q] = tr8<LDZ>(z + q * ZS, 16 * h, lane);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int h = 0; h < 8; ++h) {
          if (h + PF < 8) {
#pragma unroll
            for (int q = 0; q < 3; ++q)
              za[(h + PF) % (PF + 1)][q] = tr8<LDZ>(z + q * ZS, 16 * (h + PF), lane);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int u = 0; u < KT; ++u)
            x6_mma(za[h % (PF + 1)], xb[u][0], xb[u][1], xb[u][2], hw[h][u], lw[h][u]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if constexpr (DX) {   // after the wgrad sweep: an accumulating dX had it to arrive
#pragma unroll
        for (int u = 0; u < DT; ++u)
#pragma unroll
          for (int r = 0; r < R / 16; ++r) {
            const int64_t row = t * R + 16 * r + i;
            if (dxp[u] && row < a.n) {
              float4 v = make_float4(x6_out(dh[u][r][0], dl[u][r][0]), x6_out(dh[u][r][1], dl[u][r][1]),
                                     x6_out(dh[u][r][2], dl[u][r][2]), x6_out(dh[u][r][3], dl[u][r][3]));
              if constexpr (ACC) {
                if (acc_dx[u]) {
                  v.x = dxo[u][r].x + v.x; v.y = dxo[u][r].y + v.y; v.z = dxo[u][r].z + v.z;
                  v.w = dxo[u][r].w + v.w;
                }
              }
              *reinterpret_cast<float4*>(dxp[u] + row * dxld[u] + 4 * g) = v;
            }
          }
      }
      if constexpr (!LATE) put(t + G, b ^ 1);
      __syncthreads();
    }
  };
  if (w >= 4) {
    loop(std::true_type{});
  } else {
    loop(std::false_type{});
  }
  if constexpr (WG) {
    // the slab row: [h][K + 1] of its own, or a column block of a shared [h][slab_ld] (the
    // K = 384 / 512 column blocks, one reduce for both)
    const int64_t KEXT = a.slab_ld > 0 ? a.slab_ld : K + 1;
    const int c0 = a.slab_ld > 0 ? a.slab_c0 : 0;
    const int64_t dbc = KEXT - 1;
    float* slab = a.slab + (int64_t)bid * kH * KEXT;
#pragma unroll
    for (int h = 0; h < 8; ++h)
#pragma unroll
      for (int u = 0; u < KT; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          slab[(int64_t)(16 * h + 4 * g + j) * KEXT + c0 + 16 * (KT * w + u) + i] =
              hw[h][u][j] + lw[h][u][j];
    // db: the 16 row groups' column partials, summed in a fixed order (the loop's last barrier
    // retired every plane read, so the planes hold the reduction)
    float4* red = reinterpret_cast<float4*>(&zp[0][0]);
    red[threadIdx.x] = dbacc;
    __syncthreads();
    if (threadIdx.x < 32) {
      float4 s = red[threadIdx.x];
#pragma unroll
      for (int q = 1; q < 16; ++q) {
        const float4 v = red[q * 32 + threadIdx.x];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      const int c = 4 * threadIdx.x;
      // (both column blocks write the same db partials: the same dz tiles in the same order)
      slab[(int64_t)(c + 0) * KEXT + dbc] = s.x;
      slab[(int64_t)(c + 1) * KEXT + dbc] = s.y;
      slab[(int64_t)(c + 2) * KEXT + dbc] = s.z;
      slab[(int64_t)(c + 3) * KEXT + dbc] = s.w;
    }
  }
}

template <int K, bool DX, bool WG, bool ACC>
__global__ void __launch_bounds__(kThr, 1) k_lin_bwd_xs(const LinArgs a, const ChunkTab tab,
                                                        int64_t n_tiles) {
  lin_bwd_xs_body<K, DX, WG, ACC>(a, tab, n_tiles, blockIdx.x, gridDim.x);
}

template <int K, bool DX, bool WG, bool ACC>
__global__ void __launch_bounds__(kThr, 1) k_lin_bwd_xs2(const XsPair p) {
  // one copy of the body: the job index is uniform (from blockIdx), so its arguments are scalar
  // loads at a uniform offset (two inlined copies spilled the K = 256 wgrad variant)
  const int j = blockIdx.x < (uint32_t)p.g0 ? 0 : 1;
  const uint32_t g0 = (uint32_t)p.g0;
  const uint32_t bid = j ? blockIdx.x - g0 : blockIdx.x;
  const uint32_t G = j ? gridDim.x - g0 : g0;
  lin_bwd_xs_body<K, DX, WG, ACC>(p.a[j], p.tab[j], p.n_tiles[j], bid, G);
}

}  // namespace

int64_t xs_bwd_grid(int64_t n_rows) {
  return std::max<int64_t>(1, std::min<int64_t>(cdiv(n_rows, 32), 256));
}

// the forward's grid: at least kFwdTilesPerBlock tiles per block (each block splits its W slice
// once; at cfg5's ~48k-row blocks 8 tiles per block: 0.631 / 0.633 vs 0.635 / 0.637 ms per batch,
// 16: 0.652; blocks of a million rows and more fill the 256 CUs either way)
constexpr int64_t kFwdTilesPerBlock = 8;
static int64_t xs_fwd_grid(int64_t n_tiles) {
  return std::max<int64_t>(1, std::min<int64_t>(cdiv(n_tiles, kFwdTilesPerBlock), 256));
}

int xs_linear_fwd(const LinArgs& a, const ChunkTab& tab, hipStream_t stream) {
  if (a.n >= (int64_t(1) << 31)) return fail(HGNN_E_UNSUPPORTED, "k_lin_fwd_xs: n >= 2^31 rows");
  const int K = a.k_total;
  const int64_t R = K == 256 ? 32 : 64;
  const int64_t n_tiles = cdiv(a.n, R);
  const dim3 grid((unsigned)xs_fwd_grid(n_tiles)), block(kThr);
  if (K == 128) {
    if (a.add) hipLaunchKernelGGL((k_lin_fwd_xs<128, true>), grid, block, 0, stream, a, tab, n_tiles);
    else hipLaunchKernelGGL((k_lin_fwd_xs<128, false>), grid, block, 0, stream, a, tab, n_tiles);
  } else {
    if (a.add) hipLaunchKernelGGL((k_lin_fwd_xs<256, true>), grid, block, 0, stream, a, tab, n_tiles);
    else hipLaunchKernelGGL((k_lin_fwd_xs<256, false>), grid, block, 0, stream, a, tab, n_tiles);
  }
  return check_launch("k_lin_fwd_xs");
}

// A two-job launch's grids: each job's own grid, scaled to one chip's worth (256 blocks, one per
// CU) in tile proportion when they add up to more — the two jobs then run side by side instead of
// the second waiting for the first's blocks.
static void pair_grids(int64_t t0, int64_t t1, int64_t g0, int64_t g1, int64_t (&g)[2]) {
  g[0] = g0;
  g[1] = g1;
  if (g0 + g1 > 256) {
    g[0] = std::max<int64_t>(1, std::min<int64_t>(g0, (256 * t0 + (t0 + t1) / 2) / (t0 + t1)));
    g[1] = std::max<int64_t>(1, std::min<int64_t>(g1, 256 - g[0]));
  }
}

int xs_linear_fwd2(const LinArgs (&a)[2], const ChunkTab (&tab)[2], hipStream_t stream) {
  if (a[0].n >= (int64_t(1) << 31) || a[1].n >= (int64_t(1) << 31))
    return fail(HGNN_E_UNSUPPORTED, "k_lin_fwd_xs2: n >= 2^31 rows");
  const int K = a[0].k_total;
  const int64_t R = K == 256 ? 32 : 64;
  XsPair p;
  int64_t g[2], own[2];
  for (int j = 0; j < 2; ++j) {
    p.a[j] = a[j];
    p.tab[j] = tab[j];
    p.n_tiles[j] = cdiv(a[j].n, R);
    own[j] = xs_fwd_grid(p.n_tiles[j]);
  }
  pair_grids(p.n_tiles[0], p.n_tiles[1], own[0], own[1], g);
  p.g0 = g[0];
  const dim3 grid((unsigned)(g[0] + g[1])), block(kThr);
  const bool add = a[0].add != nullptr;
  if (K == 128) {
    if (add) hipLaunchKernelGGL((k_lin_fwd_xs2<128, true>), grid, block, 0, stream, p);
    else hipLaunchKernelGGL((k_lin_fwd_xs2<128, false>), grid, block, 0, stream, p);
  } else {
    if (add) hipLaunchKernelGGL((k_lin_fwd_xs2<256, true>), grid, block, 0, stream, p);
    else hipLaunchKernelGGL((k_lin_fwd_xs2<256, false>), grid, block, 0, stream, p);
  }
  return check_launch("k_lin_fwd_xs2");
}

int xs_bwd_class(const LinArgs& a, const ChunkTab& tab, bool dx) {
  bool acc = false;
  for (int c = 0; c < a.k_total / 16; ++c) acc |= tab.dx[c] && ((tab.dx_acc >> c) & 1u);
  return (dx ? 1 : 0) | (a.slab ? 2 : 0) | (acc && dx ? 4 : 0);
}

int xs_linear_bwd2(const LinArgs (&a)[2], const ChunkTab (&tab)[2], bool dx, int (&grid_out)[2],
                   hipStream_t stream) {
  if (a[0].n >= (int64_t(1) << 31) || a[1].n >= (int64_t(1) << 31))
    return fail(HGNN_E_UNSUPPORTED, "k_lin_bwd_xs2: n >= 2^31 rows");
  const int K = a[0].k_total;
  const int cls = xs_bwd_class(a[0], tab[0], dx);
  if (cls != xs_bwd_class(a[1], tab[1], dx) || K != a[1].k_total)
    return fail(HGNN_E_ARG, "k_lin_bwd_xs2: the two jobs differ in K or variant");
  XsPair p;
  int64_t g[2];
  for (int j = 0; j < 2; ++j) {
    p.a[j] = a[j];
    p.tab[j] = tab[j];
    p.n_tiles[j] = cdiv(a[j].n, 32);
  }
  pair_grids(p.n_tiles[0], p.n_tiles[1], xs_bwd_grid(a[0].n), xs_bwd_grid(a[1].n), g);
  p.g0 = g[0];
  grid_out[0] = (int)g[0];
  grid_out[1] = (int)g[1];
  const bool wg = (cls & 2) != 0, acc = (cls & 4) != 0;
  const dim3 grid((unsigned)(g[0] + g[1])), block(kThr);
#define HGNN_BXS2(KV, DXV, WGV, ACCV) \
  hipLaunchKernelGGL((k_lin_bwd_xs2<KV, DXV, WGV, ACCV>), grid, block, 0, stream, p)
  if (K == 128 && dx) {
    if (wg) { if (acc) HGNN_BXS2(128, true, true, true); else HGNN_BXS2(128, true, true, false); }
    else { if (acc) HGNN_BXS2(128, true, false, true); else HGNN_BXS2(128, true, false, false); }
  } else if (K == 128) {
    HGNN_BXS2(128, false, true, false);
  } else {
    if (dx) {
      if (acc) HGNN_BXS2(256, true, false, true); else HGNN_BXS2(256, true, false, false);
      if (int rc = check_launch("k_lin_bwd_xs2")) return rc;
    }
    if (wg) {
      p.a[0].dz_out = p.a[1].dz_out = nullptr;   // the dgrad pass wrote it
      HGNN_BXS2(256, false, true, false);
    }
  }
#undef HGNN_BXS2
  return check_launch("k_lin_bwd_xs2");
}

int xs_linear_bwd(const LinArgs& a, const ChunkTab& tab, bool dx, int* grid_out,
                  hipStream_t stream) {
  if (a.n >= (int64_t(1) << 31)) return fail(HGNN_E_UNSUPPORTED, "k_lin_bwd_xs: n >= 2^31 rows");
  const int K = a.k_total;
  const int64_t n_tiles = cdiv(a.n, 32);
  const int64_t G = xs_bwd_grid(a.n);
  *grid_out = (int)G;
  const bool wg = a.slab != nullptr;
  const dim3 grid((unsigned)G), block(kThr);
  bool acc = false;
  for (int c = 0; c < K / 16; ++c) acc |= tab.dx[c] && ((tab.dx_acc >> c) & 1u);
#define HGNN_BXS(KV, DXV, WGV, ACCV) \
  hipLaunchKernelGGL((k_lin_bwd_xs<KV, DXV, WGV, ACCV>), grid, block, 0, stream, a, tab, n_tiles)
  if (K == 128 && dx) {
    if (wg) { if (acc) HGNN_BXS(128, true, true, true); else HGNN_BXS(128, true, true, false); }
    else { if (acc) HGNN_BXS(128, true, false, true); else HGNN_BXS(128, true, false, false); }
  } else if (K == 128) {
    HGNN_BXS(128, false, true, false);
  } else {
    // K = 256: the dgrad and the wgrad as two passes (their registers do not fit one wave)
    if (dx) {
      if (acc) HGNN_BXS(256, true, false, true); else HGNN_BXS(256, true, false, false);
      if (int rc = check_launch("k_lin_bwd_xs")) return rc;
    }
    if (wg) {
      LinArgs b = a;
      b.dz_out = nullptr;   // the dgrad pass wrote it
      hipLaunchKernelGGL((k_lin_bwd_xs<256, false, true, false>), grid, block, 0, stream, b, tab,
                         n_tiles);
    }
  }
#undef HGNN_BXS
  return check_launch("k_lin_bwd_xs");
}

}  // namespace hgnn
