// Probe: the K3 forward tile (N = 9M rows, K = H = 128, out = relu(x W^T + b)) on bf16 MFMA with
// an fp32-exact split ("bf16x6"): x = x1 + x2 + x3 and w = w1 + w2 + w3 (each piece the bf16
// rounding of what the previous pieces leave), out = sum of the six products whose pieces' orders
// add to <= 4 (x1w1 | x1w2 + x2w1 + x1w3 + x3w1 + x2w2; the dropped terms are ~2^-24 of |x||w|),
// the large product and the five small ones in separate f32 accumulators.  v_mfma_f32_16x16x32_bf16
// (16 cycles, 16x16x32) against the f32 path's v_mfma_f32_16x16x4_f32 (32 cycles, 16x16x4): per
// 16 x 16 x 128 output tile 24 x 16 = 384 MFMA cycles instead of 32 x 32 = 1024.
// W's three planes are split once per block into LDS (3 x 128 x 136 bf16 = 104 KB, one block of
// 8 waves per CU); each wave streams 16-row tiles, splitting its X fragments in registers.
// Reports ms, TF/s (of the f32 GEMM's 2NKH) and the max error against double on sampled rows,
// next to the f32-MFMA probe kernel of k3_probe.hip's structure.
//   hipcc -O3 --offload-arch=gfx950 scripts/k3_x6_probe.hip -o /tmp/k3_x6 && /tmp/k3_x6
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned short bf16_bits(float f) {
  return __bfloat16_as_ushort(__float2bfloat16(f));   // round to nearest even
}
__device__ __forceinline__ float bf16_val(unsigned short b) {
  return __uint_as_float(((unsigned)b) << 16);
}

// three bf16 pieces of 8 floats
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& p1, bf16x8& p2, bf16x8& p3) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const unsigned short a = bf16_bits(x[j]);
    const float r1 = x[j] - bf16_val(a);
    const unsigned short b = bf16_bits(r1);
    const float r2 = r1 - bf16_val(b);
    p1[j] = (short)a;
    p2[j] = (short)b;
    p3[j] = (short)bf16_bits(r2);
  }
}

constexpr int H = 128, K = 128, NT = H / 16, KS = K / 32, LDB = K + 8;   // bf16 row stride

// WAVES waves per block (one block per CU: the W planes take 104 KB); ACC2: the big product and
// the five small ones in separate accumulators (else one)
template <int WAVES, bool ACC2, bool MEMONLY = false>
__global__ void __launch_bounds__(64 * WAVES, 1) k_x6(const float* __restrict__ x,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ bias, float* out,
                                                      int64_t n, int64_t n_tiles) {
  __shared__ __attribute__((aligned(16))) unsigned short wp[3][H * LDB];
  for (int idx = threadIdx.x; idx < H * K; idx += 64 * WAVES) {
    const int j = idx / K, k = idx % K;
    const float v = w[idx];
    const unsigned short a = bf16_bits(v);
    const float r1 = v - bf16_val(a);
    const unsigned short b = bf16_bits(r1);
    wp[0][j * LDB + k] = a;
    wp[1][j * LDB + k] = b;
    wp[2][j * LDB + k] = bf16_bits(r1 - bf16_val(b));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int64_t nw = (int64_t)gridDim.x * WAVES;
  const int64_t last = n - 1;
  int64_t t = (int64_t)blockIdx.x * WAVES + wave;
  // this lane's X: row i of the tile, k = 32 s + 8 g .. +7 for s = 0..3 (8 float4)
  float4 xv[KS][2];
  auto load_s = [&](int64_t tt, int s) {
    const int64_t row = min<int64_t>(tt * 16 + i, last);
    const float4* p = reinterpret_cast<const float4*>(x + row * K + 32 * s + 8 * g);
    xv[s][0] = p[0];
    xv[s][1] = p[1];
  };
  if (t < n_tiles) {
#pragma unroll
    for (int s = 0; s < KS; ++s) load_s(t, s);
  }
  __syncthreads();
  for (; t < n_tiles; t += nw) {
    const int64_t tn = t + nw < n_tiles ? t + nw : t;
    // opaque per-tile LDS base: keeps the loop-invariant W fragments as LDS reads instead of
    // letting the compiler hoist all 3 x 8 x 4 of them into (spilled) registers
    int wo = i * LDB + 8 * g;
    asm volatile("" : "+v"(wo));
    f32x4 hi[NT], lo[ACC2 ? NT : 1];
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      hi[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (ACC2) lo[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // W fragments one column tile ahead (s-major order of (s, c) pairs)
    bf16x8 cw[3], nx[3];
    auto rd = [&](int s, int c, bf16x8 (&f)[3]) {
      const int off = wo + 16 * c * LDB + 32 * s;
#pragma unroll
      for (int q = 0; q < 3; ++q) f[q] = *reinterpret_cast<const bf16x8*>(&wp[q][off]);
    };
    rd(0, 0, cw);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float xf[8] = {xv[s][0].x, xv[s][0].y, xv[s][0].z, xv[s][0].w,
                     xv[s][1].x, xv[s][1].y, xv[s][1].z, xv[s][1].w};
      bf16x8 x1, x2, x3;
      split8(xf, x1, x2, x3);
      load_s(tn, s);      // the next tile's chunk s, in flight for a whole tile of MFMAs
      if constexpr (MEMONLY) {   // the loads, the split and the stores without the MFMAs
#pragma unroll
        for (int c = 0; c < NT; ++c)
          hi[c][c & 3] += __uint_as_float((unsigned)(unsigned short)x1[c] << 16) +
                          __uint_as_float((unsigned)(unsigned short)x3[c] << 16);
        continue;
      }
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        if (c + 1 < NT) rd(s, c + 1, nx);
        else if (s + 1 < KS) rd(s + 1, 0, nx);
        f32x4& L = ACC2 ? lo[ACC2 ? c : 0] : hi[c];
        L = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[1], x2, L, 0, 0, 0);
        L = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[2], x1, L, 0, 0, 0);
        L = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[0], x3, L, 0, 0, 0);
        L = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[1], x1, L, 0, 0, 0);
        L = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[0], x2, L, 0, 0, 0);
        hi[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[0], x1, hi[c], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 3; ++q) cw[q] = nx[q];
      }
    }
    const int64_t row = t * 16 + i;
    if (row < n) {
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        const float4 bb = *reinterpret_cast<const float4*>(bias + 16 * c + 4 * g);
        f32x4 a = hi[c];
        if constexpr (ACC2) a += lo[c];
        float4 v = make_float4(fmaxf(a[0] + bb.x, 0.f), fmaxf(a[1] + bb.y, 0.f),
                               fmaxf(a[2] + bb.z, 0.f), fmaxf(a[3] + bb.w, 0.f));
        *reinterpret_cast<float4*>(out + row * H + 16 * c + 4 * g) = v;
      }
    }
  }
}

__global__ void k_fill(float* p, int64_t n, uint32_t seed) {
  for (int64_t k = blockIdx.x * 256ll + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) {
    uint32_t h = (uint32_t)k * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[k] = ((int)(h & 0xffffff) - 8388608) * (1.f / 8388608.f);   // 24 random bits in [-1, 1)
  }
}

template <int WAVES, bool ACC2, bool MEMONLY = false>
static void run(const char* name, float* x, float* w, float* b, float* out, int64_t n,
                int64_t n_tiles, int grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r)
    hipLaunchKernelGGL((k_x6<WAVES, ACC2, MEMONLY>), dim3(grid), dim3(64 * WAVES), 0, 0, x, w, b, out, n,
                       n_tiles);
  hipEventRecord(e0, 0);
  const int reps = 10;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_x6<WAVES, ACC2, MEMONLY>), dim3(grid), dim3(64 * WAVES), 0, 0, x, w, b, out, n,
                       n_tiles);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  const double flops = 2.0 * n * K * H;
  // error against double on sampled rows, relative to the row's max |out|
  const int64_t rows[8] = {0, 1, 15, 16, 4097, n / 3, n / 2 + 7, n - 1};
  static float hx[K], hw[H * K], hb[H], ho[H];
  hipMemcpy(hw, w, sizeof(hw), hipMemcpyDeviceToHost);
  hipMemcpy(hb, b, sizeof(hb), hipMemcpyDeviceToHost);
  double worst = 0, worst_pre = 0;
  for (int q = 0; q < 8; ++q) {
    hipMemcpy(hx, x + rows[q] * K, sizeof(hx), hipMemcpyDeviceToHost);
    hipMemcpy(ho, out + rows[q] * H, sizeof(ho), hipMemcpyDeviceToHost);
    double ref[H], mx = 0;
    for (int j = 0; j < H; ++j) {
      double s = hb[j];
      for (int k = 0; k < K; ++k) s += (double)hx[k] * hw[j * K + k];
      ref[j] = s > 0 ? s : 0;
      mx = fmax(mx, fabs(s));
    }
    for (int j = 0; j < H; ++j) {
      worst = fmax(worst, fabs(ho[j] - ref[j]) / mx);
      double a = fabs((double)hb[j]);
      for (int k = 0; k < K; ++k) a += fabs((double)hx[k] * hw[j * K + k]);
      worst_pre = fmax(worst_pre, fabs(ho[j] - ref[j]) / (a * 5.96e-8));
    }
  }
  printf("{\"variant\": \"%s\", \"ms\": %.3f, \"TFLOP/s_f32_equiv\": %.1f, \"GB/s\": %.0f, "
         "\"max_err_rel_row_max\": %.2e, \"max_err_in_f32_ulps_of_sum_abs\": %.2f}\n",
         name, ms, flops / (ms * 1e-3) / 1e12, (double)n * (K + H) * 4 / (ms * 1e-3) / 1e9, worst,
         worst_pre);
}

int main() {
  const int64_t n = 9000000, n_tiles = (n + 15) / 16;
  float *x, *w, *b, *out;
  hipMalloc(&x, (size_t)n * K * 4);
  hipMalloc(&out, (size_t)n * H * 4);
  hipMalloc(&w, H * K * 4);
  hipMalloc(&b, H * 4);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n * K, 1u);
  hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, w, (int64_t)H * K, 2u);
  hipLaunchKernelGGL(k_fill, dim3(1), dim3(256), 0, 0, b, (int64_t)H, 3u);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = 256;
  run<8, true>("8 waves, 2 acc", x, w, b, out, n, n_tiles, grid);
  run<16, false>("16 waves, 1 acc", x, w, b, out, n, n_tiles, grid);
  run<16, false, true>("16 waves, memory only (no MFMA)", x, w, b, out, n, n_tiles, grid);
  run<8, false, true>("8 waves, memory only (no MFMA)", x, w, b, out, n, n_tiles, grid);
  return 0;
}
