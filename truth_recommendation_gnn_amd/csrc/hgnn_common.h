// Shared helpers for the hgnn HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include <stdarg.h>

#include "../../include/hgnn.h"

namespace hgnn {

constexpr int kWave = 64;   // CDNA wavefront; never 32

// Thread-local last error (hgnn_last_error_string).
void set_error(const char* fmt, ...);

inline int fail(int code, const char* fmt, ...) {
  char buf[384];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  set_error("%s", buf);
  return code;
}

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(HGNN_E_HIP, "%s: %s", what, hipGetErrorString(e));
  return HGNN_OK;
}

inline hipStream_t as_stream(hgnn_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline size_t align_up(size_t n, size_t a) { return (n + a - 1) / a * a; }

// Bump allocator over the caller's workspace (the library owns no persistent memory).
struct Workspace {
  char* base;
  size_t cap;
  size_t used = 0;
  Workspace(void* p, size_t c) : base(static_cast<char*>(p)), cap(c) {}
  template <typename T>
  T* take(size_t n) {
    size_t off = align_up(used, 256);
    used = off + n * sizeof(T);
    return used <= cap && base ? reinterpret_cast<T*>(base + off) : nullptr;
  }
};

// Row fragments: W = 4 (float4 per lane) when d % 4 == 0, else scalar.
template <int W>
struct Vec;
template <>
struct Vec<4> {
  using T = float4;
  static __device__ __forceinline__ T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  static __device__ __forceinline__ T load(const float* p) {
    return *reinterpret_cast<const float4*>(p);
  }
  // streaming (nt) load: for rows gathered once per edge
  static __device__ __forceinline__ T load_nt(const float* p) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  static __device__ __forceinline__ void store(float* p, T v) {
    *reinterpret_cast<float4*>(p) = v;
  }
  static __device__ __forceinline__ void store_nt(float* p, T v) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4{v.x, v.y, v.z, v.w}, reinterpret_cast<f4*>(p));
  }
  static __device__ __forceinline__ void fma(T& a, float w, T v) {
    a.x = fmaf(w, v.x, a.x); a.y = fmaf(w, v.y, a.y);
    a.z = fmaf(w, v.z, a.z); a.w = fmaf(w, v.w, a.w);
  }
  static __device__ __forceinline__ void add(T& a, T v) {
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  static __device__ __forceinline__ float dot(T a, T b) {
    return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
  }
  static __device__ __forceinline__ void scale(T& a, float s) {
    a.x *= s; a.y *= s; a.z *= s; a.w *= s;
  }
  static __device__ __forceinline__ T shfl_xor(T v, int m) {
    return make_float4(__shfl_xor(v.x, m, 64), __shfl_xor(v.y, m, 64), __shfl_xor(v.z, m, 64),
                       __shfl_xor(v.w, m, 64));
  }
};
template <>
struct Vec<1> {
  using T = float;
  static __device__ __forceinline__ T zero() { return 0.f; }
  static __device__ __forceinline__ T load(const float* p) { return *p; }
  static __device__ __forceinline__ T load_nt(const float* p) { return __builtin_nontemporal_load(p); }
  static __device__ __forceinline__ void store(float* p, T v) { *p = v; }
  static __device__ __forceinline__ void store_nt(float* p, T v) { __builtin_nontemporal_store(v, p); }
  static __device__ __forceinline__ void fma(T& a, float w, T v) { a = fmaf(w, v, a); }
  static __device__ __forceinline__ void add(T& a, T v) { a += v; }
  static __device__ __forceinline__ float dot(T a, T b) { return a * b; }
  static __device__ __forceinline__ void scale(T& a, float s) { a *= s; }
  static __device__ __forceinline__ T shfl_xor(T v, int m) { return __shfl_xor(v, m, 64); }
};

// Device exclusive scan of int32 counts (n entries) -> out (n+1 entries, out[n] = total).
// Workspace query with ws == nullptr.
// Sum over aligned groups of LPR lanes (power of 2), result in every lane of the group.  Within a
// 16-lane DPP row the butterfly runs on DPP moves (quad_perm xor 1 / xor 2, row_half_mirror,
// row_mirror) instead of LDS-pipe ds_bpermute; wider groups finish with shuffles.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <int LPR>
__device__ __forceinline__ float slot_sum(float s) {
  if constexpr (LPR >= 2) s += dpp_mov<0xB1>(s);    // quad_perm [1,0,3,2]
  if constexpr (LPR >= 4) s += dpp_mov<0x4E>(s);    // quad_perm [2,3,0,1]
  if constexpr (LPR >= 8) s += dpp_mov<0x141>(s);   // row_half_mirror
  if constexpr (LPR >= 16) s += dpp_mov<0x140>(s);  // row_mirror
  if constexpr (LPR >= 32) s += __shfl_xor(s, 16, 64);
  if constexpr (LPR >= 64) s += __shfl_xor(s, 32, 64);
  return s;
}

// Hardware transcendentals (v_exp_f32 / v_log_f32 / v_rcp_f32, ~1-2 ulp).  t = exp(-|x|) in
// (0, 1] serves both:  sigmoid(x) = x >= 0 ? 1/(1+t) : t/(1+t),  softplus(x) = max(x,0) + log(1+t)
__device__ __forceinline__ float exp_neg_abs(float x) { return __expf(-fabsf(x)); }
__device__ __forceinline__ float sigmoid_t(float x, float t) {
  const float r = __builtin_amdgcn_rcpf(1.f + t);
  return x >= 0.f ? r : t * r;
}

// Uniform int32 in [0, hi) of draw i: splitmix64 of seed + i * golden ratio, then the high 32 bits
// scaled by hi (hgnn_uniform_i32; the negatives sort regenerates the same draws in its first pass).
__device__ __forceinline__ int32_t uniform_draw(uint64_t seed, int64_t i, uint32_t hi) {
  uint64_t x = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (int32_t)(((x >> 32) * (uint64_t)hi) >> 32);
}

int exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t* ws_bytes,
                       hipStream_t stream);


}  // namespace hgnn
