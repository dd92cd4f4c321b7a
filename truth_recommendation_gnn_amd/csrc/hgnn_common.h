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
  static __device__ __forceinline__ void store(float* p, T v) {
    *reinterpret_cast<float4*>(p) = v;
  }
  static __device__ __forceinline__ void fma(T& a, float w, T v) {
    a.x = fmaf(w, v.x, a.x); a.y = fmaf(w, v.y, a.y);
    a.z = fmaf(w, v.z, a.z); a.w = fmaf(w, v.w, a.w);
  }
  static __device__ __forceinline__ void add(T& a, T v) {
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
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
  static __device__ __forceinline__ void store(float* p, T v) { *p = v; }
  static __device__ __forceinline__ void fma(T& a, float w, T v) { a = fmaf(w, v, a); }
  static __device__ __forceinline__ void add(T& a, T v) { a += v; }
  static __device__ __forceinline__ void scale(T& a, float s) { a *= s; }
  static __device__ __forceinline__ T shfl_xor(T v, int m) { return __shfl_xor(v, m, 64); }
};

// Device exclusive scan of int32 counts (n entries) -> out (n+1 entries, out[n] = total).
// Workspace query with ws == nullptr.
int exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t* ws_bytes,
                       hipStream_t stream);

}  // namespace hgnn
