// K3 (fused multi-segment linear) types and bf16-split helpers shared by linear.hip (the f32-input
// MFMA kernels, the general shapes and the C ABI) and linear_xs.hip (the split-once kernels).
#pragma once
#include "hgnn_common.h"

#include <hip/hip_bf16.h>

namespace hgnn {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));

struct Seg {
  const float* x;
  float* dx;
  int32_t k;
  int32_t off;
};

struct LinArgs {
  Seg seg[HGNN_MAX_SEG];
  int32_t n_seg;
  int32_t k_total;
  const float* w;
  int32_t ldw;            // W row stride in floats: k_total, or the whole W's K for a column block
                          // of it (the split kernels over K = 384 / 512 as two launches)
  const float* bias;
  const float* dout;
  const float* out_act;   // ReLU output for the backward mask (nullable)
  const uint32_t* mask_in;  // backward: the same mask as bits (hgnn_linear_fwd_mask; nullable)
  uint32_t* mask_out;       // forward: write the ReLU mask as bits (nullable)
  const float* add;       // forward: [n, h] rows added before the activation (nullable)
  float* dz_out;          // backward: the masked dz written out as well (nullable; dgrad kernels)
  uint32_t dx_acc;        // backward: bit s set = segment s's dX is added into dx, not stored
  float* out;
  float* slab;            // wgrad partials [gx][h][k_total+1]
  int32_t slab_ld;        // split kernels: the slab's row stride when > 0 ([gx][h][slab_ld], this
  int32_t slab_c0;        // launch's dW columns at slab_c0.., db at slab_ld - 1), else k_total + 1
  int64_t n;
  int32_t h;
  int32_t relu;
  int64_t rows_per_block; // wgrad
};

// H (output width) in {64, 128}, K (sum of segments) in {64, 128, 256}, every segment a multiple
// of 16 columns and float4-aligned.  Per 16-column chunk c of the concatenated input, a host-built
// table gives the segment base/stride (no per-element segment search).
constexpr int kMaxChunks = 16;   // K <= 256
struct ChunkTab {
  const float* x[kMaxChunks];
  float* dx[kMaxChunks];
  int32_t ld[kMaxChunks];
  int32_t col[kMaxChunks];   // first column of the chunk inside its segment
  uint32_t dx_acc;           // bit c set = chunk c's dX is added into dx (LinArgs::dx_acc)
};

// ReLU mask as bits (hgnn_linear_fwd_mask), in the lane layout the persistent kernels share:
// the lane (i, g) that holds columns 16 c + 4 g .. +3 (c = 0 .. H/16 - 1) of row i finds them in
// word row * 4 + g, bits 4 c .. 4 c + 3 (H <= 128, a multiple of 16): one 4-B word per lane per
// row, no cross-lane exchange in the forward, 16 B per row instead of the output's 4 H.
// Each element kept or zeroed by its bit: v_bfe_i32(word, bit, 1) is 0 or all ones, ANDed with
// the element's bits — two VALU per element, no compare, select or VCC hazard (a zeroed element
// is +0, a NaN with its bit clear too, as the select gave)
__device__ __forceinline__ float mask1(float v, uint32_t word, int bit) {
  const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)word, (unsigned)bit, 1u);
  return __uint_as_float(__float_as_uint(v) & m);
}
__device__ __forceinline__ float4 mask4(float4 v, uint32_t word, int shift) {
  v.x = mask1(v.x, word, shift);
  v.y = mask1(v.y, word, shift + 1);
  v.z = mask1(v.z, word, shift + 2);
  v.w = mask1(v.w, word, shift + 3);
  return v;
}

// ReLU as one v_max_f32 per element (fmaxf(v, 0) compiles to a canonicalize + max pair); a NaN
// gives 0, as fmaxf does
__device__ __forceinline__ float relu1(float v) {
  float r;
  asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(v));
  return r;
}
__device__ __forceinline__ float4 relu4(float4 v) {
  return make_float4(relu1(v.x), relu1(v.y), relu1(v.z), relu1(v.w));
}

__device__ __forceinline__ uint32_t relu_bits(float4 v, int shift) {
  return ((v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) |
          (v.w > 0.f ? 8u : 0u)) << shift;
}

// relu_bits of a ReLU OUTPUT (every element +0, -0 or positive; relu1 maps NaN to 0): v > 0 is
// exactly "the bits as a signed int are >= 1", so one v_med3_i32(bits, 0, 1) per element gives
// the bit and three v_lshl_or_b32 pack them — 8 VALU where the compares and selects took 11 plus
// the VCC hazard nops between them
__device__ __forceinline__ uint32_t pos_bit(float v) {
  uint32_t r;
  asm("v_med3_i32 %0, %1, 0, 1" : "=v"(r) : "v"(v));
  return r;
}
__device__ __forceinline__ uint32_t relu_out_bits(float4 v, int shift) {
  uint32_t r = pos_bit(v.x) << shift;
  r |= pos_bit(v.y) << (shift + 1);
  r |= pos_bit(v.z) << (shift + 2);
  r |= pos_bit(v.w) << (shift + 3);
  return r;
}

// dX fragment store of the persistent kernels: stored, or added into what dx holds (the
// gradient of a node table that another update already wrote — one pass instead of a torch add)
__device__ __forceinline__ void store_dx4(float* p, bool add, float a0, float a1, float a2,
                                          float a3) {
  float4* q = reinterpret_cast<float4*>(p);
  if (add) {
    const float4 o = *q;
    *q = make_float4(o.x + a0, o.y + a1, o.z + a2, o.w + a3);
  } else {
    *q = make_float4(a0, a1, a2, a3);
  }
}

// ================================================================ bf16x6: fp32-exact split
// gfx950 runs bf16 MFMA at 16x the fp32 MFMA rate (2.5 PF vs 157 TF dense).  Every fp32 value
// v splits exactly-enough into three bf16 pieces, v1 = bf16(v), v2 = bf16(v - v1),
// v3 = bf16(v - v1 - v2) (|v - v1 - v2 - v3| <= ~2^-24 |v|), and a product x w becomes the six
// piece products whose orders add to <= 4: x1w1 | x1w2 + x2w1 + x1w3 + x3w1 + x2w2 (the dropped
// x2w3, x3w2, x3w3 are <= ~2^-24 |x w|).  Each piece product is exact in f32 and accumulates in
// f32, so the result has fp32 accuracy: measured at most 0.68 f32 ulp of sum |x w| against
// double (scripts/k3_x6_probe.hip; the large product and the five small ones kept in separate
// accumulators), with v_mfma_f32_16x16x32_bf16 (16 cycles per 16x16x32) doing 24 MFMAs per
// 16 x 16 x 128 tile where the f32 form needs 32 of v_mfma_f32_16x16x4_f32 at 32 cycles.
// Non-finite values: v1 = bf16(v) carries an inf (or NaN) into the large product, whose
// accumulator holds nothing else; the residual pieces of an inf are NaN (inf - inf), so the small
// products' accumulator turns NaN (as it may from an inf times W's mixed-sign residual pieces),
// and x6_out takes a large-product sum of +-inf as the result on its own.  So an inf input gives
// the +-inf (or NaN) the f32 kernels give; a finite |v| above the largest bf16 (3.39e38, which
// rounds to inf) is the one case that differs.  (Round 3 also clamped each residual to a finite
// value with a v_med3 per element; x6_out makes that redundant.)

// The split, two values at once: one v_cvt_pk_bf16_f32 per piece pair, whose packed word is already the
// operand layout (a in the low half); the pieces' f32 values are the word shifted (low half) or
// masked (high half); the residuals are exact.  (Element-wise, the compiler emits one
// convert per value plus a v_perm per pair to pack them — ~7.75 instead of 5.5 VALU per value.)
__device__ __forceinline__ uint32_t x6_cvt_pk(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ void x6_split2(float a, float b, uint32_t& p1, uint32_t& p2,
                                          uint32_t& p3) {
  p1 = x6_cvt_pk(a, b);
  const float ra = a - __uint_as_float(p1 << 16), rb = b - __uint_as_float(p1 & 0xffff0000u);
  p2 = x6_cvt_pk(ra, rb);
  const float sa = ra - __uint_as_float(p2 << 16), sb = rb - __uint_as_float(p2 & 0xffff0000u);
  p3 = x6_cvt_pk(sa, sb);
}
__device__ __forceinline__ void x6_split4(const float4& u, bf16x4_t& p1, bf16x4_t& p2,
                                          bf16x4_t& p3) {
  uint32_t a1, a2, a3, b1, b2, b3;
  x6_split2(u.x, u.y, a1, a2, a3);
  x6_split2(u.z, u.w, b1, b2, b3);
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  p1 = __builtin_bit_cast(bf16x4_t, (u32x2){a1, b1});
  p2 = __builtin_bit_cast(bf16x4_t, (u32x2){a2, b2});
  p3 = __builtin_bit_cast(bf16x4_t, (u32x2){a3, b3});
}
__device__ __forceinline__ void x6_split8(const float4& u, const float4& v, bf16x8_t& p1,
                                          bf16x8_t& p2, bf16x8_t& p3) {
  bf16x4_t a1, a2, a3, b1, b2, b3;
  x6_split4(u, a1, a2, a3);
  x6_split4(v, b1, b2, b3);
  p1 = __builtin_shufflevector(a1, b1, 0, 1, 2, 3, 4, 5, 6, 7);
  p2 = __builtin_shufflevector(a2, b2, 0, 1, 2, 3, 4, 5, 6, 7);
  p3 = __builtin_shufflevector(a3, b3, 0, 1, 2, 3, 4, 5, 6, 7);
}
// hi + lo of the split's two accumulators, hi alone when it is +-inf (see above): lo clamped to
// +-FLT_MAX by one v_med3_f32 (IEEE mode: a NaN lo yields the median of the bounds, +FLT_MAX),
// so an infinite hi survives the add and a finite hi gets its finite lo unchanged.  One
// instruction in place of the class test and select (probe: scripts/probe_minmax.hip)
__device__ __forceinline__ float x6_out(float hi, float lo) {
  float c;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(c) : "v"(lo), "v"(-0x1.fffffep127f), "v"(0x1.fffffep127f));
  return hi + c;
}

// acc_hi += w1 x1; acc_lo += w2 x2 + w3 x1 + w1 x3 + w2 x1 + w1 x2 (small terms first)
__device__ __forceinline__ void x6_mma(const bf16x8_t (&w)[3], const bf16x8_t& x1,
                                       const bf16x8_t& x2, const bf16x8_t& x3, f32x4& hi,
                                       f32x4& lo) {
  lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], x2, lo, 0, 0, 0);
  lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], x1, lo, 0, 0, 0);
  lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x3, lo, 0, 0, 0);
  lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], x1, lo, 0, 0, 0);
  lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x2, lo, 0, 0, 0);
  hi = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x1, hi, 0, 0, 0);
}

// Two jobs of one split-kernel launch (k_lin_fwd_xs2 / k_lin_bwd_xs2): blocks [0, g0) run job
// 0, the rest job 1; the jobs share K and the kernel variant.
struct XsPair {
  LinArgs a[2];
  ChunkTab tab[2];
  int64_t n_tiles[2];
  int64_t g0;
};

// The split-once kernels (linear_xs.hip): H = 128, K = 128 / 256, every segment 16-column
// chunked and float4-aligned.  Host launchers; the caller validated the arguments.
int xs_linear_fwd(const LinArgs& a, const ChunkTab& tab, hipStream_t stream);
// dW / db partials into a.slab (grid blocks x [H][K + 1]); the caller reduces them.  dx: run the
// dgrad too (tab.dx).  Returns the block count through *grid.
int xs_linear_bwd(const LinArgs& a, const ChunkTab& tab, bool dx, int* grid, hipStream_t stream);
int64_t xs_bwd_grid(int64_t n_rows);
// The same for two jobs in one launch each (the same K; in the backward the same dgrad /
// wgrad / accumulate variant); grid[j]: job j's block count (its slab rows).
int xs_linear_fwd2(const LinArgs (&a)[2], const ChunkTab (&tab)[2], hipStream_t stream);
int xs_linear_bwd2(const LinArgs (&a)[2], const ChunkTab (&tab)[2], bool dx, int (&grid)[2],
                   hipStream_t stream);
// the split kernels' backward variant of a job: bit 0 dgrad, bit 1 wgrad, bit 2 accumulate
int xs_bwd_class(const LinArgs& a, const ChunkTab& tab, bool dx);

}  // namespace hgnn
