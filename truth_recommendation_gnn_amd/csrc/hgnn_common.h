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

// Device exclusive scan of int32 counts (n entries) -> out (n+1 entries, out[n] = total).
// Workspace query with ws == nullptr.
int exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t* ws_bytes,
                       hipStream_t stream);

}  // namespace hgnn
