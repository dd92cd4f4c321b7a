// Standalone hetero epilogue (K4 on its own): out = act( sum_r w_r * in_r ), the weighted relation
// sum + ReLU of WeightedRGCN.forward (train_gnn.py:187-198), and its backward.
//
// The model path never launches these: the relation weights are folded into the K3 weight image
// and the bias/ReLU into K3's epilogue.  They exist for callers that run SAGEConv
// per relation through hgnn_linear_fwd_f32 and combine the outputs themselves — the reference's
// own call pattern.  Pure streaming: float4 grid-stride loops, HBM-bound at
// 4·(n_in + 1)·n bytes forward.
#include "hgnn_common.h"

namespace hgnn {

struct EpiArgs {
  const float* in[HGNN_MAX_SEG];
  float* din[HGNN_MAX_SEG];
  float w[HGNN_MAX_SEG];
  int n_in;
  int64_t n;        // elements
  int relu;
  const float* out;   // backward: forward output (ReLU mask)
  const float* dout;
  float* res;         // forward output
};

template <int W>
__device__ __forceinline__ typename Vec<W>::T ld(const float* p, int64_t i) {
  return Vec<W>::load(p + i * W);
}

template <int W>
__global__ void __launch_bounds__(256) k_epilogue_fwd(EpiArgs a) {
  using V = Vec<W>;
  const int64_t nv = a.n / W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv;
       i += (int64_t)gridDim.x * blockDim.x) {
    typename V::T acc = V::zero();
    for (int r = 0; r < a.n_in; ++r) V::fma(acc, a.w[r], ld<W>(a.in[r], i));
    if (a.relu) {
      if constexpr (W == 4) {
        acc.x = fmaxf(acc.x, 0.f); acc.y = fmaxf(acc.y, 0.f);
        acc.z = fmaxf(acc.z, 0.f); acc.w = fmaxf(acc.w, 0.f);
      } else {
        acc = fmaxf(acc, 0.f);
      }
    }
    V::store(a.res + i * W, acc);
  }
}

template <int W>
__global__ void __launch_bounds__(256) k_epilogue_bwd(EpiArgs a) {
  using V = Vec<W>;
  const int64_t nv = a.n / W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv;
       i += (int64_t)gridDim.x * blockDim.x) {
    typename V::T g = ld<W>(a.dout, i);
    if (a.relu) {
      const typename V::T o = ld<W>(a.out, i);
      if constexpr (W == 4) {
        g.x = o.x > 0.f ? g.x : 0.f; g.y = o.y > 0.f ? g.y : 0.f;
        g.z = o.z > 0.f ? g.z : 0.f; g.w = o.w > 0.f ? g.w : 0.f;
      } else {
        g = o > 0.f ? g : 0.f;
      }
    }
    for (int r = 0; r < a.n_in; ++r) {
      if (!a.din[r]) continue;
      typename V::T d = g;
      V::scale(d, a.w[r]);
      V::store(a.din[r] + i * W, d);
    }
  }
}

static bool aligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

static unsigned epi_grid(int64_t nv) {
  return (unsigned)std::min<int64_t>(std::max<int64_t>(cdiv(nv, 256), 1), 256 * 16);
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_hetero_epilogue(int32_t n_in, const float* const* ins, const float* weights, int64_t n,
                         int32_t relu, float* out, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_in < 1 || n_in > HGNN_MAX_SEG || n < 0 || !ins || !weights)
    return fail(HGNN_E_ARG, "hetero_epilogue: n_in=%d n=%lld", n_in, (long long)n);
  if (n == 0) return HGNN_OK;
  if (!out) return fail(HGNN_E_ARG, "hetero_epilogue: out is null");
  EpiArgs a{};
  bool vec = n % 4 == 0 && aligned16(out);
  for (int r = 0; r < n_in; ++r) {
    if (!ins[r]) return fail(HGNN_E_ARG, "hetero_epilogue: input %d is null", r);
    a.in[r] = ins[r];
    a.w[r] = weights[r];
    vec = vec && aligned16(ins[r]);
  }
  a.n_in = n_in;
  a.n = n;
  a.relu = relu;
  a.res = out;
  if (vec)
    hipLaunchKernelGGL(k_epilogue_fwd<4>, dim3(epi_grid(n / 4)), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(k_epilogue_fwd<1>, dim3(epi_grid(n)), dim3(256), 0, stream, a);
  return check_launch("k_epilogue_fwd");
}

int hgnn_hetero_epilogue_bwd(int32_t n_in, const float* weights, int64_t n, int32_t relu,
                             const float* out, const float* dout, float* const* dins,
                             hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_in < 1 || n_in > HGNN_MAX_SEG || n < 0 || !weights || !dins)
    return fail(HGNN_E_ARG, "hetero_epilogue_bwd: n_in=%d n=%lld", n_in, (long long)n);
  if (n == 0) return HGNN_OK;
  if (!dout || (relu && !out)) return fail(HGNN_E_ARG, "hetero_epilogue_bwd: null pointer");
  EpiArgs a{};
  bool vec = n % 4 == 0 && aligned16(dout) && (!relu || aligned16(out));
  for (int r = 0; r < n_in; ++r) {
    a.din[r] = dins[r];
    a.w[r] = weights[r];
    vec = vec && (!dins[r] || aligned16(dins[r]));
  }
  a.n_in = n_in;
  a.n = n;
  a.relu = relu;
  a.out = out;
  a.dout = dout;
  if (vec)
    hipLaunchKernelGGL(k_epilogue_bwd<4>, dim3(epi_grid(n / 4)), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(k_epilogue_bwd<1>, dim3(epi_grid(n)), dim3(256), 0, stream, a);
  return check_launch("k_epilogue_bwd");
}

}  // extern "C"
