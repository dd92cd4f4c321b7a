// Adam over a list of parameter tensors in ONE launch, capturable (the step count lives on the
// device and the launch advances it itself).
//
// The reference trains with torch.optim.Adam(lr=0.001) (train_gnn.py:207); the rebuilt step
// (bench.py, minibatch.CapturedStep) replays it inside the recorded graph.  torch's capturable
// fused Adam is two launches there — a multi-tensor add for the step tensors, then the update
// over 48 blocks of 12288 threads (20 us for cfg5's 264k parameters, most of it launch-bound).
// Here every block runs 1024 elements of one tensor and the last block to finish writes the new
// step, so the replay has one node and the chip's width.
//
// The arithmetic follows torch's fused kernel (ATen fused_adam_utils.cuh, the ORIGINAL mode):
// the hyper-parameters are doubles, so beta1 * m, (1 - beta1) * g, the v update, lr / bc1 and
// the eps add are evaluated in double and rounded to float where torch stores them.
#include "hgnn_common.h"

#include <algorithm>
#include <math.h>

namespace hgnn {

constexpr int kAdamMaxTensors = 32;
constexpr int kAdamPer = 4;   // elements per thread

struct AdamArgs {
  float* p[kAdamMaxTensors];
  const float* g[kAdamMaxTensors];
  float* m[kAdamMaxTensors];
  float* v[kAdamMaxTensors];
  int64_t numel[kAdamMaxTensors];
  int32_t blk[kAdamMaxTensors + 1];   // prefix sums of the tensors' block counts
  int32_t n;
  double lr, beta1, beta2, eps, weight_decay;
  float* step;        // [1] steps done so far (the launch uses step + 1)
  uint32_t* done;     // [1] blocks finished; zero between launches (the last block resets it)
  int32_t advance;    // write step + 1 when done (the last launch of a step)
};

__global__ void __launch_bounds__(256) k_adam_multi(const AdamArgs a) {
  const float t = *a.step + 1.f;
  const float bc1 = (float)(1.0 - pow(a.beta1, (double)t));
  const float bc2_sqrt = (float)sqrt(1.0 - pow(a.beta2, (double)t));
  const float step_size = (float)(a.lr / (double)bc1);
  // the block's tensor: uniform (from blockIdx), so its pointers are scalar loads — a per-element
  // search over a flat index made them per-lane and measured slower than torch's kernel
  int lo = 0, hi = a.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (a.blk[mid] <= (int)blockIdx.x) lo = mid;
    else hi = mid - 1;
  }
  lo = __builtin_amdgcn_readfirstlane(lo);
  float* __restrict__ P = a.p[lo];
  const float* __restrict__ Gr = a.g[lo];
  float* __restrict__ M = a.m[lo];
  float* __restrict__ V = a.v[lo];
  const int64_t n = a.numel[lo];
  const int64_t base = (int64_t)(blockIdx.x - a.blk[lo]) * (256 * kAdamPer);
#pragma unroll
  for (int k = 0; k < kAdamPer; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    if (i < n) {
      float p = P[i];
      float g = Gr[i];
      if (a.weight_decay != 0.0) g = (float)((double)g + (double)p * a.weight_decay);
      float m = M[i], v = V[i];
      m = (float)(a.beta1 * (double)m + (1.0 - a.beta1) * (double)g);
      v = (float)(a.beta2 * (double)v + (1.0 - a.beta2) * (double)g * (double)g);
      const float denom = (float)((double)(sqrtf(v) / bc2_sqrt) + a.eps);
      p -= step_size * m / denom;
      P[i] = p;
      M[i] = m;
      V[i] = v;
    }
  }
  if (!a.advance) return;
  // every block read the old step above; the last one to get here writes the new one
  __shared__ bool last;
  __syncthreads();
  if (threadIdx.x == 0) {
    // only the order "this block read the step, then counted itself" matters (no block reads
    // another's data): a workgroup-scope fence waits for the block's own accesses, where a
    // device-scope one would write the XCD's L2 back on every block
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    last = atomicAdd(a.done, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    *a.step = t;
    atomicExch(a.done, 0u);
  }
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_adam_multi(int32_t n_tensors, float* const* params, const float* const* grads,
                    float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                    float* step, uint32_t* done, double lr, double beta1, double beta2, double eps,
                    double weight_decay, hgnn_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  if (n_tensors < 0 || !step || !done || (n_tensors > 0 && (!params || !grads || !exp_avg ||
                                                            !exp_avg_sq || !numel)))
    return fail(HGNN_E_ARG, "adam_multi: bad arguments");
  if (n_tensors == 0) return HGNN_OK;
  for (int c0 = 0; c0 < n_tensors; c0 += kAdamMaxTensors) {   // tensors in launches of 32
    AdamArgs a{};
    a.n = std::min(kAdamMaxTensors, n_tensors - c0);
    a.blk[0] = 0;
    for (int j = 0; j < a.n; ++j) {
      const int t = c0 + j;
      if (numel[t] < 0 || (numel[t] > 0 && (!params[t] || !grads[t] || !exp_avg[t] ||
                                            !exp_avg_sq[t])))
        return fail(HGNN_E_ARG, "adam_multi: tensor %d", t);
      a.p[j] = params[t];
      a.g[j] = grads[t];
      a.m[j] = exp_avg[t];
      a.v[j] = exp_avg_sq[t];
      a.numel[j] = numel[t];
      const int64_t nb = cdiv(numel[t], 256 * kAdamPer);
      if ((int64_t)a.blk[j] + nb > (int64_t(1) << 30))
        return fail(HGNN_E_UNSUPPORTED, "adam_multi: too many elements in one launch");
      a.blk[j + 1] = a.blk[j] + (int32_t)nb;
    }
    a.lr = lr; a.beta1 = beta1; a.beta2 = beta2; a.eps = eps; a.weight_decay = weight_decay;
    a.step = step;
    a.done = done;
    a.advance = c0 + kAdamMaxTensors >= n_tensors ? 1 : 0;
    if (a.blk[a.n] == 0) {   // nothing to update: the step still advances (torch's does)
      a.blk[a.n] = 1;
    }
    const unsigned grid = (unsigned)a.blk[a.n];
    hipLaunchKernelGGL(k_adam_multi, dim3(grid), dim3(256), 0, stream, a);
    if (int rc = check_launch("k_adam_multi")) return rc;
  }
  return HGNN_OK;
}

}  // extern "C"
