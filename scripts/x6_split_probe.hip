// The fp32 -> three-bf16 split of csrc/linear_common.h in two forms, bit for bit: the residuals
// as shift/mask + subtract (round 5) and as one v_dot2c_f32_bf16 against (-1, 0) / (0, -1)
// (round 6).  Random values over the whole finite range, plus denormals, signed zeros, powers of
// two and values next to bf16 rounding ties.  Prints the mismatch count and exits non-zero on any.
//   hipcc -O3 --offload-arch=gfx950 scripts/x6_split_probe.hip -o build/x6_split_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef __bf16 b2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ void split_sub(float a, float b, uint32_t* o) {
  const uint32_t p1 = cvt(a, b);
  const float ra = a - __uint_as_float(p1 << 16), rb = b - __uint_as_float(p1 & 0xffff0000u);
  const uint32_t p2 = cvt(ra, rb);
  const float sa = ra - __uint_as_float(p2 << 16), sb = rb - __uint_as_float(p2 & 0xffff0000u);
  o[0] = p1; o[1] = p2; o[2] = cvt(sa, sb);
}
__device__ __forceinline__ float rlo(uint32_t p, float a) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b2, p), __builtin_bit_cast(b2, 0x0000BF80u), a, false);
}
__device__ __forceinline__ float rhi(uint32_t p, float b) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(b2, p), __builtin_bit_cast(b2, 0xBF800000u), b, false);
}
__device__ void split_dot(float a, float b, uint32_t* o) {
  const uint32_t p1 = cvt(a, b);
  const float ra = rlo(p1, a), rb = rhi(p1, b);
  const uint32_t p2 = cvt(ra, rb);
  const float sa = rlo(p2, ra), sb = rhi(p2, rb);
  o[0] = p1; o[1] = p2; o[2] = cvt(sa, sb);
}
__global__ void k(const uint32_t* bits, int64_t n, unsigned long long* bad, uint32_t* first) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const float a = __uint_as_float(bits[2 * i]), b = __uint_as_float(bits[2 * i + 1]);
  uint32_t x[3], y[3];
  split_sub(a, b, x);
  split_dot(a, b, y);
  if (x[0] != y[0] || x[1] != y[1] || x[2] != y[2]) {
    if (atomicAdd(bad, 1ull) == 0) {
      first[0] = bits[2 * i]; first[1] = bits[2 * i + 1];
      for (int q = 0; q < 3; ++q) { first[2 + q] = x[q]; first[5 + q] = y[q]; }
    }
  }
}
static uint64_t sm(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
int main() {
  const int64_t n = int64_t(1) << 26;
  uint32_t* h = (uint32_t*)malloc(n * 4);
  uint64_t s = 12345;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t r = sm(s);
    uint32_t v = (uint32_t)r;
    switch ((r >> 32) & 7) {
      case 0: v &= 0x807fffffu; break;                                   // denormals, +-0
      case 1: v = (v & 0x80000000u) | (uint32_t)((r >> 40) % 254 + 1) << 23; break;   // 2^k
      case 2: v = (v & 0xffff0000u) | 0x8000u; break;                    // bf16 ties
      case 3: v = (v & 0xffff0000u) | 0x7fffu; break;
      default: { const uint32_t e = (v >> 23) & 0xff; if (e == 0xff) v ^= 0x00800000u; }  // finite
    }
    h[i] = v;
  }
  uint32_t *d, *df;
  unsigned long long* db;
  hipMalloc(&d, n * 4); hipMalloc(&db, 8); hipMalloc(&df, 32);
  hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
  hipMemset(db, 0, 8);
  hipLaunchKernelGGL(k, dim3((unsigned)(n / 2 / 256)), dim3(256), 0, 0, d, n, db, df);
  unsigned long long bad = 0;
  uint32_t f[8] = {0};
  hipMemcpy(&bad, db, 8, hipMemcpyDeviceToHost);
  hipMemcpy(f, df, 32, hipMemcpyDeviceToHost);
  printf("{\"pairs\": %lld, \"mismatches\": %llu", (long long)(n / 2), bad);
  if (bad) printf(", \"first\": [\"%08x\", \"%08x\", \"sub %08x %08x %08x\", \"dot %08x %08x %08x\"]", f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7]);
  printf("}\n");
  return bad ? 1 : 0;
}
