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
#ifndef HGNN_XS_STAGGER
#define HGNN_XS_STAGGER 1
#endif
#ifndef HGNN_XS_SPLITILP
#define HGNN_XS_SPLITILP 0
#endif
#ifndef HGNN_XS_MASKMED
#define HGNN_XS_MASKMED 1
#endif
// HGNN_XS_PROBE (timing probes only, wrong results): 1 = no HBM traffic in the forward (every
// tile's loads hit the first R rows, no output stores); 2 = no MFMA sweep in the forward; 3 = as 1
// with the stores kept; 4 = the loads kept, no stores
#ifndef HGNN_XS_PROBE
#define HGNN_XS_PROBE 0
#endif

namespace hgnn {

// HGNN_XS_STAMPS (a diagnostic build only, scripts/k3_stamps.py): lane 0 of every wave of the
// first 64 blocks records s_memtime at the phase boundaries of 8 loop iterations into a buffer
// of its own, read back by hgnn_debug_xs_stamps; no output and no other code reads them.
#ifndef HGNN_XS_STAMPS
#define HGNN_XS_STAMPS 0
#endif
#if HGNN_XS_STAMPS
constexpr int kStampBlocks = 64, kStampIters = 8, kStampFirst = 40, kStampPts = 12;
__device__ unsigned long long g_xs_stamps[kStampBlocks * 8 * kStampIters * kStampPts];
#define XS_STAMP(it, k)                                                                          \
  do {                                                                                           \
    if (blockIdx.x < kStampBlocks && (it) >= kStampFirst && (it) < kStampFirst + kStampIters) {   \
      const unsigned long long ts_ = __builtin_amdgcn_s_memtime();                               \
      if ((threadIdx.x & 63) == 0)                                                               \
        g_xs_stamps[(((int)blockIdx.x * 8 + (int)(threadIdx.x >> 6)) * kStampIters +            \
                     ((it) - kStampFirst)) * kStampPts + (k)] = ts_;                            \
    }                                                                                            \
  } while (0)
// points 8 / 9: after an explicit wait for every outstanding memory operation right before the
// late / early waves' split — how much of a split phase is waiting for its loads
#define XS_WAIT_STAMP(it, k)                                                                     \
  do {                                                                                           \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                            \
    XS_STAMP(it, k);                                                                             \
  } while (0)
#else
#define XS_STAMP(it, k) do { } while (0)
#define XS_WAIT_STAMP(it, k) do { } while (0)
#endif

namespace {

constexpr int kH = 128;     // output width
constexpr int kThr = 512;   // 8 waves

typedef short v4s __attribute__((ext_vector_type(4)));

// row clamp (a mixed-type min<int64_t>(int64, int32) compiled to f64 converts and v_min_f64)
__device__ __forceinline__ uint32_t clamp_row(int64_t row, int32_t last) {
  return min((uint32_t)row, (uint32_t)last);   // row < 2^32: n < 2^31 and at most 2 G R past it
}
typedef __attribute__((address_space(3))) v4s lds_v4s;

// The three-piece split of N float4 at once, level by level (HGNN_XS_SPLITILP): every level's
// converts, extracts and subtractions are independent across the 2N value pairs, where the
// per-pair order chains ~11 dependent instructions (in-kernel stamps: a wave's split of 16
// values took ~900 cycles for ~90 VALU).  pc[level][j][h]: the packed bf16 pair of level
// `level` for values 2h, 2h+1 of float4 j — the words x6_split4 produces.
template <int N>
__device__ __forceinline__ void x6_split_levels(float (&v)[N][4], uint32_t (&pc)[3][N][2]) {
#pragma unroll
  for (int lv = 0; lv < 3; ++lv) {
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) pc[lv][j][h] = x6_cvt_pk(v[j][2 * h], v[j][2 * h + 1]);
    if (lv < 2) {
#pragma unroll
      for (int j = 0; j < N; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          v[j][2 * h] -= __uint_as_float(pc[lv][j][h] << 16);
          v[j][2 * h + 1] -= __uint_as_float(pc[lv][j][h] & 0xffff0000u);
        }
    }
  }
}
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
    const uint32_t row = (HGNN_XS_PROBE == 1 || HGNN_XS_PROBE == 3) ? (uint32_t)(row0 + j * RSTEP)
                                                                    : clamp_row(r0 + row0 + j * RSTEP, last);
    x.v[j] = *reinterpret_cast<const float4*>(base + (uint64_t)row * ld);
  }
  __device__ __forceinline__ void issue(Regs& x, int64_t r0, int32_t last) const {
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const uint32_t row = (HGNN_XS_PROBE == 1 || HGNN_XS_PROBE == 3) ? (uint32_t)(row0 + j * RSTEP)
                                              : clamp_row(r0 + row0 + j * RSTEP, last);
      x.v[j] = *reinterpret_cast<const float4*>(base + (uint64_t)row * ld);
    }
  }
  // split into the three planes (plane stride PS halfwords, row stride LDP).  ZERO: rows past n
  // (clamped copies of the last row) become zeros — the backward's reductions over rows need
  // that (0 x inf would be NaN); a forward row only reaches its own output, never stored
  template <int LDP, int PS, bool ZERO = false>
  __device__ __forceinline__ void put(const Regs& x, unsigned short* pl, int64_t r0,
                                      int64_t n = 0) const {
#if HGNN_XS_SPLITILP
    // the split level by level across all NL float4 (2 NL value pairs): each level's converts,
    // extracts and subtractions are independent, where the per-pair order chained ~11
    // dependent instructions (stamps: a wave's split took ~900 cycles for ~90 VALU)
    float v[NL][4];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      float4 u = x.v[j];
      if (ZERO && r0 + row0 + j * RSTEP >= n) u = make_float4(0.f, 0.f, 0.f, 0.f);
      v[j][0] = u.x; v[j][1] = u.y; v[j][2] = u.z; v[j][3] = u.w;
    }
    uint32_t pc[3][NL][2];
    x6_split_levels<NL>(v, pc);
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      unsigned short* d = pl + (row0 + j * RSTEP) * LDP + col;
#pragma unroll
      for (int lv = 0; lv < 3; ++lv)
        *reinterpret_cast<bf16x4_t*>(d + lv * PS) =
            __builtin_bit_cast(bf16x4_t, (xs_u32x2){pc[lv][j][0], pc[lv][j][1]});
    }
    return;
#endif
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      float4 v = x.v[j];
      if (ZERO && r0 + row0 + j * RSTEP >= n) v = make_float4(0.f, 0.f, 0.f, 0.f);
      bf16x4_t p1, p2, p3;
      x6_split4(v, p1, p2, p3);
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
// Per tile: [the previous tile's output stores] [this tile's added rows, the next tile's X]
// [MFMA sweep] [epilogue into registers] [split of the next tile into the other buffer] [barrier].
// Memory order matters because vmcnt is one in-order counter: a wait on an operation also waits
// for everything issued before it.  The outputs are stored at the top of the NEXT iteration,
// before its loads, and their registers are held until after that iteration's sweep: the
// compiler waits for a store to read its data before it lets anything overwrite those registers,
// and with the stores issued last (before the barrier) that wait landed at the loop head and
// drained the prefetch with them.  The prefetch is unconditional (past the last tile the rows
// clamp and the split goes to an unread buffer): a conditional issue made the waitcnt pass
// assume loads in flight at the loop head and wait for everything there.  (Measured and not
// kept: loads two tiles ahead in a second register set, the split interleaved into the sweep
// — 3.84 vs 3.69 ms at 9M rows, K = 256; the kernel runs at a power-limited ~1.75 GHz, so
// what counts is the instruction count, not the overlap.)
// HGNN_XS_VMEM_STEP: the sweep step after which the iteration's memory instructions are issued
// (-1: before the sweep).  In-kernel stamps (scripts/k3_stamps.py) showed each wave spending
// ~600 cycles at the top of every iteration issuing them — all 8 waves queue ~48 KB of requests
// on the CU's memory pipe right after the barrier — while its partner split: the matrix pipe sat
// idle ~670 cycles per iteration.
#ifndef HGNN_XS_VMEM_STEP
#define HGNN_XS_VMEM_STEP -1
#endif
constexpr int kVmemStep = HGNN_XS_VMEM_STEP;
#ifndef HGNN_XS_BIASINIT
#define HGNN_XS_BIASINIT 0
#endif
constexpr bool kBiasInit = HGNN_XS_BIASINIT != 0;
// HGNN_XS_VMEM_SPREAD (default on, round 5): the iteration's memory instructions one or two per
// sweep step (the added rows first, then the previous tile's stores and mask words, then the
// prefetch) instead of one burst after the barrier.  Probes (HGNN_XS_PROBE) put ~1 ms of the
// K = 256 forward's 3.45 ms in its loads and stores (no HBM traffic: 2.52 ms; stores only 2.96;
// loads only 3.12), and the stamps showed all 8 waves stalled ~600 cycles issuing them at once.
// A/B at the cfg4 shapes: K = 128 + add 2.589 -> 2.512 ms, K = 128 (preprojection, 1M rows)
// 0.219 -> 0.198, K = 256 unchanged (3.433 / 3.436).
#ifndef HGNN_XS_VMEM_SPREAD
#define HGNN_XS_VMEM_SPREAD 1
#endif
constexpr bool kSpread = HGNN_XS_VMEM_SPREAD != 0;
// (Measured and not kept: the output tile staged in LDS and stored as whole rows, 1 KiB of
// contiguous output per wave store instead of 16 rows x 64 B — K = 256 forward 3.46 -> 3.56 ms
// with the spread, 3.50 in one burst.)

template <int K, bool ADD>
__global__ void __launch_bounds__(kThr, 1) k_lin_fwd_xs(const LinArgs a, const ChunkTab tab,
                                                        int64_t n_tiles) {
  constexpr int R = K == 256 ? 32 : 64, KS = K / 32, RT = R / 16, LDP = K + 16, PS = R * LDP;
  __shared__ __attribute__((aligned(16))) unsigned short pl[2][3 * PS];
  __shared__ uint32_t mk[2][R * 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int32_t last = (int32_t)(a.n - 1);
  const int64_t G = gridDim.x;
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
  auto store_one = [&](int64_t tp, int r) {
    const int64_t row = tp * R + 16 * r + i;
    if (HGNN_XS_PROBE != 1 && HGNN_XS_PROBE != 4 && row < a.n)
      *reinterpret_cast<float4*>(a.out + row * kH + 16 * w + 4 * g) = po[r];
  };
  auto mask_one = [&](int64_t tp, int bp) {
    if (mask_out && threadIdx.x < R * 4) {
      const int64_t row = tp * R + (threadIdx.x >> 2);
      if (HGNN_XS_PROBE != 1 && HGNN_XS_PROBE != 4 && row < a.n)
        a.mask_out[tp * R * 4 + threadIdx.x] = mk[bp][threadIdx.x];
      mk[bp][threadIdx.x] = 0u;
    }
  };
  auto store_prev = [&](int64_t tp, int bp) {
#pragma unroll
    for (int r = 0; r < RT; ++r) store_one(tp, r);
    if (mask_out && threadIdx.x < R * 4) {   // its mask words are complete (last barrier)
      const int64_t row = tp * R + (threadIdx.x >> 2);
      if (HGNN_XS_PROBE != 1 && HGNN_XS_PROBE != 4 && row < a.n) a.mask_out[tp * R * 4 + threadIdx.x] = mk[bp][threadIdx.x];
      mk[bp][threadIdx.x] = 0u;
    }
  };
  int64_t t = blockIdx.x;   // the grid never exceeds n_tiles
  xs.issue(xr, t * R, last);
  xs.template put<LDP, PS>(xr, pl[0], t * R);
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
  // (Measured and not kept: a prefetch two tiles deep in a second register set, with the added
  // rows one tile ahead too — the 9M-row launches unchanged, 3.63 vs 3.66 ms at K = 256; round 5
  // again for the early waves only, the loop unrolled by two so the sets alternate at compile
  // time: 3.575 / 3.574 ms at K = 256, 2.614 / 2.613 at K = 128 + add.)
  auto loop = [&](auto late_c) {
    constexpr bool LATE = decltype(late_c)::value;
    if constexpr (LATE) xs.issue(xr, (t + G) * R, last);
    __syncthreads();
    int it = 0;
    for (; t < n_tiles; t += G, ++it) {
      const int b = it & 1;
      XS_STAMP(it, 0);
      if constexpr (LATE) XS_WAIT_STAMP(it, 8);
      if constexpr (LATE) xs.template put<LDP, PS>(xr, pl[b ^ 1], (t + G) * R);
      XS_STAMP(it, 1);
      // the iteration's memory instructions: the previous tile's output stores, this tile's
      // added rows, the prefetch
      auto vmem = [&]() {
        if (it > 0) store_prev(t - G, b ^ 1);
        if constexpr (ADD) {
#pragma unroll
          for (int r = 0; r < RT; ++r) {
            const uint32_t row = (HGNN_XS_PROBE == 1 || HGNN_XS_PROBE == 3) ? (uint32_t)(16 * r + i)
                                                    : clamp_row(t * R + 16 * r + i, last);
            ad[r] = *reinterpret_cast<const float4*>(a.add + (uint64_t)row * kH + 16 * w + 4 * g);
          }
          __builtin_amdgcn_sched_barrier(0);   // issued before the prefetch: waited for alone
        }
        xs.issue(xr, (t + (LATE ? 2 : 1) * G) * R, last);
        __builtin_amdgcn_sched_barrier(0);   // keep the loads ahead of what follows
      };
      // the same instructions spread over the sweep (HGNN_XS_VMEM_SPREAD): piece k at step
      // k * NQ / NP — the added rows, the stores, the mask words, the prefetch
      auto vmem_step = [&](int q) {
        constexpr int NA = ADD ? RT : 0, NX = XStage<K, R>::NL, NP = NA + RT + 1 + NX;
        constexpr int NQ = RT * (K / 32);
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          if (k * NQ / NP != q) continue;
          if (k < NA) {
            if constexpr (ADD) {
              const uint32_t row = (HGNN_XS_PROBE == 1 || HGNN_XS_PROBE == 3)
                                       ? (uint32_t)(16 * k + i)
                                       : clamp_row(t * R + 16 * k + i, last);
              ad[k] = *reinterpret_cast<const float4*>(a.add + (uint64_t)row * kH + 16 * w + 4 * g);
            }
          } else if (k < NA + RT) {
            if (it > 0) store_one(t - G, k - NA);
          } else if (k == NA + RT) {
            if (it > 0) mask_one(t - G, b ^ 1);
          } else {
            xs.issue_one(xr, (t + (LATE ? 2 : 1) * G) * R, last, k - NA - RT - 1);
          }
        }
      };
      if constexpr (kVmemStep < 0 && !kSpread) vmem();
      XS_STAMP(it, 2);
      const unsigned short* p = pl[b];
      f32x4 hi[RT], lo[RT];
#if HGNN_XS_LDSPF
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
          // HGNN_XS_BIASINIT: the bias as the large-term accumulator's initial value (a GEMM
          // with C = bias), not an add per element in the epilogue
          hi[r] = kBiasInit ? f32x4{bb.x, bb.y, bb.z, bb.w} : f32x4{0.f, 0.f, 0.f, 0.f};
          lo[r] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int q = 0; q < PF; ++q) ld(q, fr[q]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          if constexpr (kVmemStep >= 0) {
            if (q == kVmemStep) vmem();   // after the sweep has the matrix pipe going
          }
          if constexpr (kSpread) vmem_step(q);
          if (q + PF < NQ) ld(q + PF, fr[(q + PF) % (PF + 1)]);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (HGNN_XS_PROBE != 2)
            x6_mma(wa[q % KS], fr[q % (PF + 1)][0], fr[q % (PF + 1)][1], fr[q % (PF + 1)][2],
                   hi[q / KS], lo[q / KS]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#else
      static_assert(!kSpread, "HGNN_XS_VMEM_SPREAD needs HGNN_XS_LDSPF");
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        hi[r] = kBiasInit ? f32x4{bb.x, bb.y, bb.z, bb.w} : f32x4{0.f, 0.f, 0.f, 0.f};
        lo[r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const bf16x8_t x1 = row8<LDP>(p, 16 * r, 32 * s, i, g);
          const bf16x8_t x2 = row8<LDP>(p + PS, 16 * r, 32 * s, i, g);
          const bf16x8_t x3 = row8<LDP>(p + 2 * PS, 16 * r, 32 * s, i, g);
          x6_mma(wa[s], x1, x2, x3, hi[r], lo[r]);
        }
      }
#endif
      XS_STAMP(it, 3);
      // the stored rows' registers are reserved until here (see above)
#pragma unroll
      for (int r = 0; r < RT; ++r)
        asm volatile("" ::"v"(po[r].x), "v"(po[r].y), "v"(po[r].z), "v"(po[r].w));
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        float4 v;
        if constexpr (kBiasInit) {
          v = make_float4(x6_out(hi[r][0], lo[r][0]), x6_out(hi[r][1], lo[r][1]),
                          x6_out(hi[r][2], lo[r][2]), x6_out(hi[r][3], lo[r][3]));
        } else {
          v = make_float4(x6_out(hi[r][0], lo[r][0]) + bb.x, x6_out(hi[r][1], lo[r][1]) + bb.y,
                          x6_out(hi[r][2], lo[r][2]) + bb.z, x6_out(hi[r][3], lo[r][3]) + bb.w);
        }
        if constexpr (ADD) {
          v.x += ad[r].x; v.y += ad[r].y; v.z += ad[r].z; v.w += ad[r].w;
        }
        if (a.relu) v = relu4(v);
        po[r] = v;
#if HGNN_XS_MASKMED
        if (mask_out) atomicOr(&mk[b][(16 * r + i) * 4 + g], relu_out_bits(v, 4 * w));
#else
        if (mask_out) atomicOr(&mk[b][(16 * r + i) * 4 + g], relu_bits(v, 4 * w));
#endif
      }
      XS_STAMP(it, 4);
      if constexpr (!LATE) XS_WAIT_STAMP(it, 9);
      if constexpr (!LATE) xs.template put<LDP, PS>(xr, pl[b ^ 1], (t + G) * R);
      XS_STAMP(it, 5);
      __syncthreads();
      XS_STAMP(it, 6);
    }
    store_prev(t - G, (it - 1) & 1);
  };
#if HGNN_XS_STAGGER
  if (w >= 4) {
    loop(std::true_type{});
  } else {
    loop(std::false_type{});
  }
#else
  loop(std::false_type{});
#endif
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
__global__ void __launch_bounds__(kThr, 1) k_lin_bwd_xs(const LinArgs a, const ChunkTab tab,
                                                        int64_t n_tiles) {
  static_assert(!(DX && WG) || K == 128, "dgrad + wgrad in one pass: K = 128");
  constexpr int R = 32, LDZ = kH + 16, LDX = K + 16, ZS = R * LDZ, XS = R * LDX;
  constexpr int KT = K / 128;      // 16-column k tiles of dW per wave
  constexpr int HS = kH / 32;      // dgrad MFMA k-steps (reduction over h)
  __shared__ __attribute__((aligned(16))) unsigned short zp[2][3 * ZS];
  __shared__ __attribute__((aligned(16))) unsigned short xp[WG ? 2 : 1][WG ? 3 * XS : 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int32_t last32 = (int32_t)(a.n - 1);
  const int64_t G = gridDim.x;
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
  auto put = [&](int64_t tt, int b, int sit) {   // sit: the iteration for stamp 10 / 11, or -1
#if HGNN_XS_SPLITILP
    float zs[ZL][4];
#endif
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
#if HGNN_XS_SPLITILP
      zs[j][0] = z.x; zs[j][1] = z.y; zs[j][2] = z.z; zs[j][3] = z.w;
    }
    {
      uint32_t pc[3][ZL][2];
      x6_split_levels<ZL>(zs, pc);
#pragma unroll
      for (int j = 0; j < ZL; ++j) {
        unsigned short* d = zp[b] + (zr + 16 * j) * LDZ + zc;
#pragma unroll
        for (int lv = 0; lv < 3; ++lv)
          *reinterpret_cast<bf16x4_t*>(d + lv * ZS) =
              __builtin_bit_cast(bf16x4_t, (xs_u32x2){pc[lv][j][0], pc[lv][j][1]});
      }
#else
      bf16x4_t p1, p2, p3;
      x6_split4(z, p1, p2, p3);
      unsigned short* d = zp[b] + (zr + 16 * j) * LDZ + zc;
      *reinterpret_cast<bf16x4_t*>(d) = p1;
      *reinterpret_cast<bf16x4_t*>(d + ZS) = p2;
      *reinterpret_cast<bf16x4_t*>(d + 2 * ZS) = p3;
#endif
    }
    XS_STAMP(sit, 10);
    if constexpr (WG) xs.template put<LDX, XS, true>(xr, xp[b], tt * R, a.n);
    XS_STAMP(sit, 11);
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
  int64_t t = blockIdx.x;   // the grid never exceeds n_tiles
  issue(t);
  put(t, 0, -1);
  // staggered halves as in the forward: waves 4-7 put the next tile first, then sweep
  auto loop = [&](auto late_c) {
    constexpr bool LATE = decltype(late_c)::value;
    if constexpr (LATE) issue(t + G);
    __syncthreads();
    for (int it = 0; t < n_tiles; t += G, ++it) {
      const int b = it & 1;
      XS_STAMP(it, 0);
      if constexpr (LATE) XS_WAIT_STAMP(it, 8);
      if constexpr (LATE) put(t + G, b ^ 1, it);
      XS_STAMP(it, 1);
      // an accumulating dX reads what the rows hold first: issued before the prefetch, so its
      // wait leaves the prefetch in flight
      float4 dxo[DT][ACC ? R / 16 : 1];
      auto vmem = [&]() {
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
      };
      // the memory instructions before the first sweep, or inside it (HGNN_XS_VMEM_STEP, see the
      // forward): in the dgrad sweep when there is one, else in the wgrad sweep
      if constexpr (kVmemStep < 0) vmem();
      XS_STAMP(it, 2);
      const unsigned short* z = zp[b];
      f32x4 dh[DT][DX ? R / 16 : 1], dl[DT][DX ? R / 16 : 1];
#if HGNN_XS_LDSPF
      // the sweeps software-pipelined as in the forward: each step's fragments are read PF
      // steps ahead, pinned by scheduling barriers
      // the fused dgrad + wgrad kernels are at the register limit: fewer fragments ahead there
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
          if constexpr (kVmemStep >= 0) {
            if (q == kVmemStep) vmem();
          }
          if (q + PF < NQ) ld(q + PF, fr[(q + PF) % (PF + 1)]);
          __builtin_amdgcn_sched_barrier(0);
          const bf16x8_t(&f)[3] = fr[q % (PF + 1)];
#pragma unroll
          for (int u = 0; u < DT; ++u)
            x6_mma(wt[u][q % HS], f[0], f[1], f[2], dh[u][q / HS], dl[u][q / HS]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      XS_STAMP(it, 3);
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
          if constexpr (kVmemStep >= 0 && !DX) {
            if (h == (kVmemStep < 8 ? kVmemStep : 7)) vmem();
          }
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
#else
      if constexpr (DX) {
#pragma unroll
        for (int r = 0; r < R / 16; ++r) {
#pragma unroll
          for (int u = 0; u < DT; ++u) dh[u][r] = dl[u][r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < HS; ++s) {
            const bf16x8_t x1 = row8<LDZ>(z, 16 * r, 32 * s, i, g);
            const bf16x8_t x2 = row8<LDZ>(z + ZS, 16 * r, 32 * s, i, g);
            const bf16x8_t x3 = row8<LDZ>(z + 2 * ZS, 16 * r, 32 * s, i, g);
#pragma unroll
            for (int u = 0; u < DT; ++u) x6_mma(wt[u][s], x1, x2, x3, dh[u][r], dl[u][r]);
          }
        }
      }
      if constexpr (WG) {
        const unsigned short* x = xp[b];
        bf16x8_t xb[KT][3];
#pragma unroll
        for (int u = 0; u < KT; ++u)
#pragma unroll
          for (int q = 0; q < 3; ++q) xb[u][q] = tr8<LDX>(x + q * XS, 16 * (KT * w + u), lane);
#pragma unroll
        for (int h = 0; h < 8; ++h) {
          bf16x8_t za[3];
#pragma unroll
          for (int q = 0; q < 3; ++q) za[q] = tr8<LDZ>(z + q * ZS, 16 * h, lane);
#pragma unroll
          for (int u = 0; u < KT; ++u) x6_mma(za, xb[u][0], xb[u][1], xb[u][2], hw[h][u], lw[h][u]);
        }
      }
#endif
      XS_STAMP(it, 4);
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
      XS_STAMP(it, 5);
      if constexpr (!LATE) XS_WAIT_STAMP(it, 9);
      if constexpr (!LATE) put(t + G, b ^ 1, -1);
      XS_STAMP(it, 6);
      __syncthreads();
      XS_STAMP(it, 7);
    }
  };
#if HGNN_XS_STAGGER
  if (w >= 4) {
    loop(std::true_type{});
  } else {
    loop(std::false_type{});
  }
#else
  loop(std::false_type{});
#endif
  if constexpr (WG) {
    // the slab row: [h][K + 1] of its own, or a column block of a shared [h][slab_ld] (the
    // K = 384 / 512 column blocks, one reduce for both)
    const int64_t KEXT = a.slab_ld > 0 ? a.slab_ld : K + 1;
    const int c0 = a.slab_ld > 0 ? a.slab_c0 : 0;
    const int64_t dbc = KEXT - 1;
    float* slab = a.slab + (int64_t)blockIdx.x * kH * KEXT;
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

}  // namespace

#if HGNN_XS_STAMPS
extern "C" int hgnn_debug_xs_stamps(unsigned long long* host, size_t n) {
  const size_t have = sizeof(g_xs_stamps) / sizeof(g_xs_stamps[0]);
  if (n > have) n = have;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_xs_stamps), n * sizeof(unsigned long long)) ==
                 hipSuccess ? (int)n : -1;
}
#endif

int64_t xs_bwd_grid(int64_t n_rows) {
  return std::max<int64_t>(1, std::min<int64_t>(cdiv(n_rows, 32), 256));
}

int xs_linear_fwd(const LinArgs& a, const ChunkTab& tab, hipStream_t stream) {
  if (a.n >= (int64_t(1) << 31)) return fail(HGNN_E_UNSUPPORTED, "k_lin_fwd_xs: n >= 2^31 rows");
  const int K = a.k_total;
  const int64_t R = K == 256 ? 32 : 64;
  const int64_t n_tiles = cdiv(a.n, R);
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(n_tiles, 256))), block(kThr);
  if (K == 128) {
    if (a.add) hipLaunchKernelGGL((k_lin_fwd_xs<128, true>), grid, block, 0, stream, a, tab, n_tiles);
    else hipLaunchKernelGGL((k_lin_fwd_xs<128, false>), grid, block, 0, stream, a, tab, n_tiles);
  } else {
    if (a.add) hipLaunchKernelGGL((k_lin_fwd_xs<256, true>), grid, block, 0, stream, a, tab, n_tiles);
    else hipLaunchKernelGGL((k_lin_fwd_xs<256, false>), grid, block, 0, stream, a, tab, n_tiles);
  }
  return check_launch("k_lin_fwd_xs");
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
