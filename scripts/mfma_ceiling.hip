// The fp32 MFMA ceiling on this box, for K3's roofline: back-to-back
// v_mfma_f32_16x16x4_f32 (the instruction K3 issues) on every SIMD of every CU, operands in
// registers, ACC independent accumulator chains per wave, W waves per SIMD.  Reports TF/s
// against the 157.3 TF/s spec and the shader clock the chip ran at (s_memtime cycles per wave /
// the wave's s_memrealtime span at 100 MHz).
//   hipcc -O3 --offload-arch=gfx950 scripts/mfma_ceiling.hip -o /tmp/mfma_ceiling && /tmp/mfma_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int ACC>
__global__ void __launch_bounds__(256) k_mfma_loop(int iters, float seed, float* out,
                                                   unsigned long long* clk) {
  f32x4 c[ACC];
#pragma unroll
  for (int q = 0; q < ACC; ++q) c[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = seed + threadIdx.x * 1e-7f, b = seed - threadIdx.x * 1e-7f;
  const unsigned long long t0 = clock64(), r0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int q = 0; q < ACC; ++q) c[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[q], 0, 0, 0);
  }
  const unsigned long long t1 = clock64(), r1 = wall_clock64();
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < ACC; ++q) s += c[q][0] + c[q][1] + c[q][2] + c[q][3];
  if (s == 12345.f) out[threadIdx.x] = s;   // keep the chain alive
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    clk[2 * w] = t1 - t0;
    clk[2 * w + 1] = r1 - r0;
  }
}

template <int ACC>
static void run(int blocks_per_cu, int iters) {
  const int cus = 256, blocks = cus * blocks_per_cu, waves = blocks * 4;
  float* out;
  unsigned long long* clk;
  hipMalloc(&out, 1024 * 4);
  hipMalloc(&clk, (size_t)waves * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k_mfma_loop<ACC>, dim3(blocks), dim3(256), 0, 0, iters / 10, 1.f, out, clk);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_mfma_loop<ACC>, dim3(blocks), dim3(256), 0, 0, iters, 1.f, out, clk);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long* h = (unsigned long long*)malloc((size_t)waves * 16);
  hipMemcpy(h, clk, (size_t)waves * 16, hipMemcpyDeviceToHost);
  double cyc = 0, real = 0;
  for (int w = 0; w < waves; ++w) {
    cyc += (double)h[2 * w];
    real += (double)h[2 * w + 1];
  }
  const double ghz = cyc / (real / 100e6) / 1e9;   // s_memrealtime runs at 100 MHz
  const double flops = (double)waves * iters * 8 * ACC * 2.0 * 16 * 16 * 4;
  printf("{\"acc_chains\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"TFLOP/s\": %.1f, "
         "\"frac_of_157.3\": %.3f, \"shader_GHz\": %.3f}\n",
         ACC, blocks_per_cu, ms, flops / (ms * 1e-3) / 1e12, flops / (ms * 1e-3) / 157.3e12, ghz);
  free(h);
  hipFree(out);
  hipFree(clk);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  run<4>(1, iters);
  run<4>(2, iters);
  run<8>(1, iters);
  run<8>(2, iters);
  run<2>(2, iters);
  return 0;
}
