// Round 6 probe (not part of the library): the fp32 -> three-bf16 split of csrc/linear_common.h
// with the low value's residual a - lo(p) as one v_dot2c_f32_bf16 (p dotted with the bf16 pair
// (-1, 0), accumulated onto a; the constant kept in a VGPR the compiler cannot fold), against the
// shift + subtract form, bit for bit over 2^25 pairs (random finite values, denormals, signed
// zeros, powers of two, bf16 rounding ties, some inf / NaN).  Result (profiles/
// r6_x6_split_probe.json): every mismatch involves an input that is, or rounds to, a bf16 inf or
// NaN.  But the same residual inside the K3 split kernels failed the K3 parity tests (K = 256 at
// n = 1, half the outputs wrong), so the form is NOT used.  Earlier
// forms, also here for the record: the constant folded by hipcc into an inline -1.0 / literal
// operand of v_dot2c (read by the hardware as the pair (0, -1) / truncated: every pair wrong),
// and the VOP3P v_dot2_f32_bf16 through inline asm (garbage); the high value's residual with the
// pair (0, -1) came out as b unchanged.
//   hipcc -O3 --offload-arch=gfx950 scripts/x6_split_probe.hip -o /tmp/x6_split_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
  asm("" : "+v"(v));
  return v;
}
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float rlo(uint32_t p, float a) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, p),
                                         __builtin_bit_cast(bf16x2, opaque(0x0000BF80u)), a, false);
}
__device__ __forceinline__ float rhi(uint32_t p, float b) { return b - __uint_as_float(p & 0xffff0000u); }
__device__ void split_dot(float a, float b, uint32_t* o) {
  const uint32_t p1 = cvt(a, b);
  const float ra = rlo(p1, a), rb = rhi(p1, b);
  const uint32_t p2 = cvt(ra, rb);
  const float sa = rlo(p2, ra), sb = rhi(p2, rb);
  o[0] = p1; o[1] = p2; o[2] = cvt(sa, sb);
}
// an inf or NaN, or a finite value at or above the bf16 overflow threshold
__device__ __forceinline__ bool nonfinite(uint32_t v) { return (v & 0x7fffffffu) >= 0x7f7f8000u; }
// cls[0]: mismatches; [1]: with an input of the class above (expected); [2]: others (fail)
__global__ void k(const uint32_t* bits, int64_t n, unsigned long long* cls, uint32_t* first) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const uint32_t ua = bits[2 * i], ub = bits[2 * i + 1];
  uint32_t x[3], y[3];
  split_sub(__uint_as_float(ua), __uint_as_float(ub), x);
  split_dot(__uint_as_float(ua), __uint_as_float(ub), y);
  if (x[0] != y[0] || x[1] != y[1] || x[2] != y[2]) {
    atomicAdd(&cls[0], 1ull);
    const int c = (nonfinite(ua) || nonfinite(ub)) ? 1 : 2;
    if (atomicAdd(&cls[c], 1ull) == 0) {
      uint32_t* f = first + c * 8;
      f[0] = ua; f[1] = ub;
      for (int q = 0; q < 3; ++q) { f[2 + q] = x[q]; f[5 + q] = y[q]; }
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
      case 0: v &= 0x807fffffu; break;                                                  // denormals
      case 1: v = (v & 0x80000000u) | (uint32_t)((r >> 40) % 254 + 1) << 23; break;     // 2^k
      case 2: v = (v & 0xffff0000u) | 0x8000u; break;                                   // ties
      case 3: v = (v & 0xffff0000u) | 0x7fffu; break;
      default: break;
    }
    h[i] = v;
  }
  uint32_t *d, *df;
  unsigned long long* db;
  if (hipMalloc(&d, n * 4) || hipMalloc(&db, 3 * 8) || hipMalloc(&df, 3 * 8 * 4)) return 2;
  if (hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice) || hipMemset(db, 0, 3 * 8) ||
      hipMemset(df, 0, 3 * 8 * 4)) return 2;
  hipLaunchKernelGGL(k, dim3((unsigned)(n / 2 / 256)), dim3(256), 0, 0, d, n, db, df);
  unsigned long long cls[3] = {0};
  uint32_t f[3 * 8] = {0};
  if (hipMemcpy(cls, db, sizeof(cls), hipMemcpyDeviceToHost) ||
      hipMemcpy(f, df, sizeof(f), hipMemcpyDeviceToHost)) return 2;
  printf("{\"pairs\": %lld, \"mismatches\": %llu, \"with_bf16_nonfinite_input\": %llu, "
         "\"other\": %llu}\n", (long long)(n / 2), cls[0], cls[1], cls[2]);
  return cls[2] ? 1 : 0;
}
