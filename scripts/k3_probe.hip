// What bounds the K3 forward at the cfg4 user-side shape (N = 9M, K = H = 128)?  The v5 kernel's
// structure (persistent, W image in LDS, k-step-major NT accumulators, next tile's X chunk loaded
// as the current one is consumed, bias + ReLU + float4 stores) with the memory sides switched off
// one at a time:
//   real   : X rows from HBM, output stored (the kernel as shipped, minus the mask bits)
//   x_l2   : X rows from a 1024-row window (L2-resident), output stored
//   nostore: X rows from HBM, output not stored (kept alive by a predicated store never taken)
//   none   : neither
// Each reports ms, TF/s and the shader clock (s_memtime cycles / s_memrealtime span, as in
// mfma_ceiling.hip), so a slower variant can be split into clock and issue.
//   hipcc -O3 --offload-arch=gfx950 scripts/k3_probe.hip -o /tmp/k3_probe && /tmp/k3_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <math.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <bool REALX, bool STORE>
__global__ void __launch_bounds__(512, 2) k_probe(const float* __restrict__ x,
                                                  const float* __restrict__ w,
                                                  const float* __restrict__ bias, float* out,
                                                  int64_t n, int64_t n_tiles, int never,
                                                  unsigned long long* clk) {
  constexpr int H = 128, K = 128, NT = H / 16, KC = K / 16, LDW = K + 8;
  __shared__ __attribute__((aligned(16))) float ws[H * LDW];
  for (int idx = threadIdx.x; idx < H * K / 4; idx += 512) {
    const int j = idx / (K / 4), k = (idx % (K / 4)) * 4;
    *reinterpret_cast<float4*>(ws + j * LDW + k) =
        *reinterpret_cast<const float4*>(w + (int64_t)j * K + k);
  }
  const unsigned long long t0 = clock64(), r0 = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int64_t nw = (int64_t)gridDim.x * 8;
  const int64_t last = n - 1;
  auto src = [&](int64_t t, int c) {
    int64_t row = min<int64_t>(t * 16 + i, last);
    if (!REALX) row &= 1023;
    return reinterpret_cast<const float4*>(x + row * K + c * 16 + 4 * g);
  };
  int64_t t = (int64_t)blockIdx.x * 8 + wave;
  float4 av[KC];
  if (t < n_tiles) {
#pragma unroll
    for (int c = 0; c < KC; ++c) av[c] = *src(t, c);
  }
  __syncthreads();
  const int wl0 = i * LDW + 4 * g;
  float keep = 0.f;
  for (; t < n_tiles; t += nw) {
    const int64_t tn = t + nw < n_tiles ? t + nw : t;
    int wo = wl0;
    asm volatile("" : "+v"(wo));
    const float* wl = ws + wo;
    const int64_t row = t * 16 + i;
    f32x4 acc[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 bw[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) bw[tt] = *reinterpret_cast<const float4*>(wl + tt * 16 * LDW);
#pragma unroll
    for (int c = 0; c < KC; ++c) {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) acc[tt] = mfma4(bw[tt].x, av[c].x, acc[tt]);
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) acc[tt] = mfma4(bw[tt].y, av[c].y, acc[tt]);
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) acc[tt] = mfma4(bw[tt].z, av[c].z, acc[tt]);
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        acc[tt] = mfma4(bw[tt].w, av[c].w, acc[tt]);
        if (c + 1 < KC)
          bw[tt] = *reinterpret_cast<const float4*>(wl + tt * 16 * LDW + (c + 1) * 16);
      }
      av[c] = *src(tn, c);
    }
    if (row < n) {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        const float4 bb = *reinterpret_cast<const float4*>(bias + tt * 16 + 4 * g);
        float4 v = make_float4(fmaxf(acc[tt][0] + bb.x, 0.f), fmaxf(acc[tt][1] + bb.y, 0.f),
                               fmaxf(acc[tt][2] + bb.z, 0.f), fmaxf(acc[tt][3] + bb.w, 0.f));
        if (STORE || never)
          *reinterpret_cast<float4*>(out + row * H + tt * 16 + 4 * g) = v;
        else
          keep += v.x + v.y + v.z + v.w;
      }
    }
  }
  if (keep == 12345.f) out[threadIdx.x] = keep;
  const unsigned long long t1 = clock64(), r1 = wall_clock64();
  if (lane == 0) {
    const int wv = blockIdx.x * 8 + wave;
    clk[2 * wv] = t1 - t0;
    clk[2 * wv + 1] = r1 - r0;
  }
}

// The same tile work on v_mfma_f32_32x32x2_f32: 32-row tiles, 4 column tiles of 32, each MFMA
// (4096 flop, 16 passes) fed by one W and one X value per lane — half the operand VGPR reads and
// LDS bytes per flop of the 16x16x4 form.  Lane (i, h) = (l % 32, l / 32) supplies k = 8c + 4h + s
// at step s of chunk c (a float4 of its row), and ends with rows' out columns 32t + 8b + 4h .. +3.
typedef float f32x16 __attribute__((ext_vector_type(16)));
template <bool REALX, bool STORE>
__global__ void __launch_bounds__(512, 1) k_probe32(const float* __restrict__ x,
                                                    const float* __restrict__ w,
                                                    const float* __restrict__ bias, float* out,
                                                    int64_t n, int64_t n_tiles, int never,
                                                    unsigned long long* clk) {
  constexpr int H = 128, K = 128, NT = H / 32, KC = K / 8, LDW = K + 4;
  __shared__ __attribute__((aligned(16))) float ws[H * LDW];
  for (int idx = threadIdx.x; idx < H * K / 4; idx += 512) {
    const int j = idx / (K / 4), k = (idx % (K / 4)) * 4;
    *reinterpret_cast<float4*>(ws + j * LDW + k) =
        *reinterpret_cast<const float4*>(w + (int64_t)j * K + k);
  }
  const unsigned long long t0 = clock64(), r0 = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int64_t nw = (int64_t)gridDim.x * 8;
  const int64_t last = n - 1;
  const int64_t n32 = (n + 31) / 32;
  auto src = [&](int64_t t, int c) {
    int64_t row = min<int64_t>(t * 32 + i, last);
    if (!REALX) row &= 1023;
    return reinterpret_cast<const float4*>(x + row * K + c * 8 + 4 * h);
  };
  int64_t t = (int64_t)blockIdx.x * 8 + wave;
  float4 av[KC];
  if (t < n32) {
#pragma unroll
    for (int c = 0; c < KC; ++c) av[c] = *src(t, c);
  }
  __syncthreads();
  const int wl0 = i * LDW + 4 * h;
  float keep = 0.f;
  for (; t < n32; t += nw) {
    const int64_t tn = t + nw < n32 ? t + nw : t;
    int wo = wl0;
    asm volatile("" : "+v"(wo));
    const float* wl = ws + wo;
    const int64_t row = t * 32 + i;
    f32x16 acc[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[tt][v] = 0.f;
    float4 bw[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) bw[tt] = *reinterpret_cast<const float4*>(wl + tt * 32 * LDW);
#pragma unroll
    for (int c = 0; c < KC; ++c) {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
        acc[tt] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[tt].x, av[c].x, acc[tt], 0, 0, 0);
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
        acc[tt] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[tt].y, av[c].y, acc[tt], 0, 0, 0);
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
        acc[tt] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[tt].z, av[c].z, acc[tt], 0, 0, 0);
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        acc[tt] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[tt].w, av[c].w, acc[tt], 0, 0, 0);
        if (c + 1 < KC)
          bw[tt] = *reinterpret_cast<const float4*>(wl + tt * 32 * LDW + (c + 1) * 8);
      }
      av[c] = *src(tn, c);
    }
    if (row < n) {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int col = tt * 32 + 8 * b + 4 * h;
          const float4 bb = *reinterpret_cast<const float4*>(bias + col);
          float4 v = make_float4(fmaxf(acc[tt][4 * b] + bb.x, 0.f), fmaxf(acc[tt][4 * b + 1] + bb.y, 0.f),
                                 fmaxf(acc[tt][4 * b + 2] + bb.z, 0.f), fmaxf(acc[tt][4 * b + 3] + bb.w, 0.f));
          if (STORE || never)
            *reinterpret_cast<float4*>(out + row * H + col) = v;
          else
            keep += v.x + v.y + v.z + v.w;
        }
    }
  }
  if (keep == 12345.f) out[threadIdx.x] = keep;
  const unsigned long long t1 = clock64(), r1 = wall_clock64();
  if (lane == 0) {
    const int wv = blockIdx.x * 8 + wave;
    clk[2 * wv] = t1 - t0;
    clk[2 * wv + 1] = r1 - r0;
  }
}

// one float of out = relu(x w^T + b) in double, for the correctness line
static double ref_elem(const float* hx, const float* hw, const float* hb, int64_t r, int j) {
  double s = hb[j];
  for (int k = 0; k < 128; ++k) s += (double)hx[r * 128 + k] * hw[j * 128 + k];
  return s > 0 ? s : 0;
}

__global__ void k_fill(float* p, int64_t n, uint32_t seed) {
  for (int64_t k = blockIdx.x * 256ll + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) {
    uint32_t h = (uint32_t)k * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[k] = ((int)(h & 0xffff) - 32768) * (1.f / 32768.f);   // uniform in [-1, 1): real MFMA power
  }
}

typedef void (*ProbeFn)(const float*, const float*, const float*, float*, int64_t, int64_t, int,
                        unsigned long long*);
static void run(ProbeFn kern, int grid, const char* name, const float* x, const float* w,
                const float* b, float* out, int64_t n, unsigned long long* clk,
                unsigned long long* hclk) {
  const int64_t n_tiles = (n + 15) / 16;
  const int waves = grid * 8;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r)
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, x, w, b, out, n, n_tiles, 0, clk);
  const int reps = 10;
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, x, w, b, out, n, n_tiles, 0, clk);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  hipMemcpy(hclk, clk, (size_t)waves * 16, hipMemcpyDeviceToHost);
  double cyc = 0, real = 0;
  for (int v = 0; v < waves; ++v) {
    cyc += (double)hclk[2 * v];
    real += (double)hclk[2 * v + 1];
  }
  const double flops = 2.0 * n * 128 * 128;
  printf("{\"variant\": \"%s\", \"ms\": %.3f, \"TFLOP/s\": %.1f, \"frac_of_155.1\": %.3f, "
         "\"shader_GHz\": %.3f}\n",
         name, ms, flops / (ms * 1e-3) / 1e12, flops / (ms * 1e-3) / 155.1e12,
         cyc / (real / 100e6) / 1e9);
}

int main() {
  const int64_t n = 9000000;
  float *x, *w, *b, *out;
  unsigned long long* clk;
  hipMalloc(&x, (size_t)n * 128 * 4);
  hipMalloc(&out, (size_t)n * 128 * 4);
  hipMalloc(&w, 128 * 128 * 4);
  hipMalloc(&b, 128 * 4);
  hipMalloc(&clk, 4096 * 16);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n * 128, 1u);
  hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, w, (int64_t)128 * 128, 2u);
  hipLaunchKernelGGL(k_fill, dim3(1), dim3(256), 0, 0, b, (int64_t)128, 3u);
  unsigned long long* hclk = (unsigned long long*)malloc(4096 * 16);
  run(k_probe<true, true>, 512, "real", x, w, b, out, n, clk, hclk);
  run(k_probe<false, true>, 512, "x_l2", x, w, b, out, n, clk, hclk);
  run(k_probe<true, false>, 512, "nostore", x, w, b, out, n, clk, hclk);
  run(k_probe<false, false>, 512, "none", x, w, b, out, n, clk, hclk);
  run(k_probe32<true, true>, 256, "real32", x, w, b, out, n, clk, hclk);
  {  // correctness of the 32x32 form on sampled rows (its output is in `out` now)
    const int64_t rows[6] = {0, 1, 31, 4096 + 17, n / 2 + 5, n - 1};
    float* hx = (float*)malloc(128 * 4 * 6);
    float* hw = (float*)malloc(128 * 128 * 4);
    float hb[128], ho[128];
    hipMemcpy(hw, w, 128 * 128 * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hb, b, 128 * 4, hipMemcpyDeviceToHost);
    double worst = 0;
    for (int q = 0; q < 6; ++q) {
      hipMemcpy(hx, x + rows[q] * 128, 128 * 4, hipMemcpyDeviceToHost);
      hipMemcpy(ho, out + rows[q] * 128, 128 * 4, hipMemcpyDeviceToHost);
      for (int j = 0; j < 128; ++j) {
        const double r = ref_elem(hx, hw, hb, 0, j), d = fabs(ho[j] - r) / (fabs(r) + 1.0);
        if (d > worst) worst = d;
      }
    }
    printf("{\"real32_max_err\": %.3e}\n", worst);
  }
  run(k_probe32<false, true>, 256, "x_l2_32", x, w, b, out, n, clk, hclk);
  run(k_probe32<true, false>, 256, "nostore32", x, w, b, out, n, clk, hclk);
  run(k_probe32<false, false>, 256, "none32", x, w, b, out, n, clk, hclk);
  run(k_probe<true, true>, 512, "real", x, w, b, out, n, clk, hclk);
  run(k_probe32<true, true>, 256, "real32", x, w, b, out, n, clk, hclk);
  return 0;
}
