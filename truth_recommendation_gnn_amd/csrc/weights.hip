// The relation-weighted fused weight of one destination update, and its adjoint.
//
// WeightedRGCN's `relu(w_direct * conv_a(...) + w_social * conv_b(...))` (train_gnn.py:187-198)
// becomes ONE K3 over [aggr_1 .. aggr_R, x_dst] with
//   W = [s_1 Wl_1 | ... | s_R Wl_R | sum_r s_r Wr_r],   b = sum_r s_r bl_r.
// Built per step from the parameters (they change every step), in one launch instead of a chain of
// torch cat / mul / add kernels; the backward splits dW / db back into every parameter's gradient in
// one launch.  Products and sums are rounded separately (no fma contraction), in relation order,
// so both are bitwise what the torch expression gives.
#include "hgnn_common.h"

#include <algorithm>

namespace hgnn {

constexpr int kMaxRel = HGNN_MAX_SEG - 1;

struct FuseArgs {
  const float* wl[kMaxRel];
  const float* wr[kMaxRel];
  const float* bl[kMaxRel];
  float* dwl[kMaxRel];
  float* dwr[kMaxRel];
  float* dbl[kMaxRel];
  float scale[kMaxRel];
  int32_t k[kMaxRel];
  int32_t off[kMaxRel];
  int32_t n_rel;
  int32_t k_root;   // 0: no root block
  int32_t k_tot;
  int32_t h;
};

__device__ __forceinline__ void fuse_one(const FuseArgs& a, float* w, float* b, int64_t idx) {
#pragma clang fp contract(off)   // s_r * W_r and the sum rounded separately, as torch does
  const int64_t n = (int64_t)a.h * a.k_tot;
  if (idx < n) {
    const int j = (int)(idx / a.k_tot), c = (int)(idx % a.k_tot);
    const int root0 = a.off[a.n_rel - 1] + a.k[a.n_rel - 1];
    float v = 0.f;
    if (c < root0) {
      int r = 0;
      while (r + 1 < a.n_rel && c >= a.off[r + 1]) ++r;
      v = (a.scale[r] * a.wl[r][(int64_t)j * a.k[r] + (c - a.off[r])]);
    } else {
      const int cr = c - root0;
      bool first = true;
      for (int r = 0; r < a.n_rel; ++r) {
        if (!a.wr[r]) continue;
        const float t = (a.scale[r] * a.wr[r][(int64_t)j * a.k_root + cr]);
        v = first ? t : (v + t);
        first = false;
      }
    }
    w[idx] = v;
  } else if (b && idx < n + a.h) {
    const int j = (int)(idx - n);
    float v = 0.f;
    bool first = true;
    for (int r = 0; r < a.n_rel; ++r) {
      if (!a.bl[r]) continue;
      const float t = (a.scale[r] * a.bl[r][j]);
      v = first ? t : (v + t);
      first = false;
    }
    b[j] = v;
  }
}

__global__ void k_fuse_weights(const FuseArgs a, float* w, float* b) {
  fuse_one(a, w, b, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

__device__ __forceinline__ void split_one(const FuseArgs& a, const float* dw, const float* db,
                                          int64_t idx) {
#pragma clang fp contract(off)
  const int64_t n = (int64_t)a.h * a.k_tot;
  if (idx < n) {
    const int j = (int)(idx / a.k_tot), c = (int)(idx % a.k_tot);
    const int root0 = a.off[a.n_rel - 1] + a.k[a.n_rel - 1];
    const float g = dw[idx];
    if (c < root0) {
      int r = 0;
      while (r + 1 < a.n_rel && c >= a.off[r + 1]) ++r;
      if (a.dwl[r]) a.dwl[r][(int64_t)j * a.k[r] + (c - a.off[r])] = (g * a.scale[r]);
    } else {
      const int cr = c - root0;
      for (int r = 0; r < a.n_rel; ++r)
        if (a.dwr[r]) a.dwr[r][(int64_t)j * a.k_root + cr] = (g * a.scale[r]);
    }
  } else if (db && idx < n + a.h) {
    const int j = (int)(idx - n);
    const float g = db[j];
    for (int r = 0; r < a.n_rel; ++r)
      if (a.dbl[r]) a.dbl[r][j] = (g * a.scale[r]);
  }
}

__global__ void k_split_weight_grads(const FuseArgs a, const float* dw, const float* db) {
  split_one(a, dw, db, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// Several destination updates' fused weights (or their adjoints) in one launch: blockIdx.y is
// the update — a layer's updates are independent, so a layer costs one launch each way.
constexpr int kMaxFuseGroups = 4;
struct FuseMulti {
  FuseArgs g[kMaxFuseGroups];
  float* w[kMaxFuseGroups];
  float* b[kMaxFuseGroups];
  const float* dw[kMaxFuseGroups];
  const float* db[kMaxFuseGroups];
};

__global__ void k_fuse_weights_multi(const FuseMulti m) {
  const int g = blockIdx.y;
  fuse_one(m.g[g], m.w[g], m.b[g], (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

__global__ void k_split_weight_grads_multi(const FuseMulti m) {
  const int g = blockIdx.y;
  split_one(m.g[g], m.dw[g], m.db[g], (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

static int fill(FuseArgs& a, int32_t n_rel, const int32_t* k, int32_t k_root, const float* scale,
                int32_t h) {
  if (n_rel < 1 || n_rel > kMaxRel || h < 1 || k_root < 0 || !k || !scale)
    return fail(HGNN_E_ARG, "fuse_weights: n_rel=%d h=%d k_root=%d", n_rel, h, k_root);
  a.n_rel = n_rel;
  a.k_root = k_root;
  a.h = h;
  int32_t off = 0;
  for (int r = 0; r < n_rel; ++r) {
    if (k[r] < 1) return fail(HGNN_E_ARG, "fuse_weights: k[%d]=%d", r, k[r]);
    a.k[r] = k[r];
    a.off[r] = off;
    a.scale[r] = scale[r];
    off += k[r];
  }
  a.k_tot = off + k_root;
  return HGNN_OK;
}

}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_fuse_weights(int32_t n_rel, const float* const* wl, const int32_t* k,
                      const float* const* wr, int32_t k_root, const float* const* bl,
                      const float* scale, int32_t h, float* w_out, float* b_out,
                      hgnn_stream_t stream) {
  FuseArgs a{};
  if (int rc = fill(a, n_rel, k, k_root, scale, h)) return rc;
  if (!wl || !w_out) return fail(HGNN_E_ARG, "fuse_weights: null pointer");
  bool any_root = false, any_b = false;
  for (int r = 0; r < n_rel; ++r) {
    if (!wl[r]) return fail(HGNN_E_ARG, "fuse_weights: wl[%d] is null", r);
    a.wl[r] = wl[r];
    a.wr[r] = wr ? wr[r] : nullptr;
    a.bl[r] = bl ? bl[r] : nullptr;
    any_root |= a.wr[r] != nullptr;
    any_b |= a.bl[r] != nullptr;
  }
  if (any_root != (k_root > 0))
    return fail(HGNN_E_ARG, "fuse_weights: k_root=%d with%s root weights", k_root,
                any_root ? "" : "out");
  if (b_out && !any_b) return fail(HGNN_E_ARG, "fuse_weights: b_out without biases");
  const int64_t total = (int64_t)h * a.k_tot + (b_out ? h : 0);
  hipLaunchKernelGGL(k_fuse_weights, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     as_stream(stream), a, w_out, b_out);
  return check_launch("k_fuse_weights");
}

int hgnn_split_weight_grads(int32_t n_rel, const float* dw, const float* db, const int32_t* k,
                            int32_t k_root, const float* scale, int32_t h, float* const* dwl,
                            float* const* dwr, float* const* dbl, hgnn_stream_t stream) {
  FuseArgs a{};
  if (int rc = fill(a, n_rel, k, k_root, scale, h)) return rc;
  if (!dw) return fail(HGNN_E_ARG, "split_weight_grads: dw is null");
  for (int r = 0; r < n_rel; ++r) {
    a.dwl[r] = dwl ? dwl[r] : nullptr;
    a.dwr[r] = dwr ? dwr[r] : nullptr;
    a.dbl[r] = dbl ? dbl[r] : nullptr;
    if (a.dwr[r] && k_root == 0)
      return fail(HGNN_E_ARG, "split_weight_grads: dwr[%d] without a root block", r);
  }
  const int64_t total = (int64_t)h * a.k_tot + (db ? h : 0);
  hipLaunchKernelGGL(k_split_weight_grads, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     as_stream(stream), a, dw, db);
  return check_launch("k_split_weight_grads");
}

// The multi-update forms: group g owns the flattened per-relation entries [base_g, base_g +
// n_rel[g]) of wl / k / wr / bl / scale (and dwl / dwr / dbl).
int hgnn_fuse_weights_multi(int32_t n_groups, const int32_t* n_rel, const float* const* wl,
                            const int32_t* k, const float* const* wr, const int32_t* k_root,
                            const float* const* bl, const float* scale, int32_t h,
                            float* const* w_out, float* const* b_out, hgnn_stream_t stream) {
  if (n_groups < 1 || n_groups > kMaxFuseGroups || !n_rel || !wl || !k || !k_root || !w_out)
    return fail(HGNN_E_ARG, "fuse_weights_multi: n_groups=%d (1..%d)", n_groups, kMaxFuseGroups);
  FuseMulti m{};
  int64_t total = 1;
  for (int g = 0, base = 0; g < n_groups; base += n_rel[g], ++g) {
    FuseArgs& a = m.g[g];
    if (int rc = fill(a, n_rel[g], k + base, k_root[g], scale + base, h)) return rc;
    bool any_root = false, any_b = false;
    for (int r = 0; r < n_rel[g]; ++r) {
      if (!wl[base + r]) return fail(HGNN_E_ARG, "fuse_weights_multi: group %d wl[%d] null", g, r);
      a.wl[r] = wl[base + r];
      a.wr[r] = wr ? wr[base + r] : nullptr;
      a.bl[r] = bl ? bl[base + r] : nullptr;
      any_root |= a.wr[r] != nullptr;
      any_b |= a.bl[r] != nullptr;
    }
    m.w[g] = w_out[g];
    m.b[g] = b_out ? b_out[g] : nullptr;
    if (!m.w[g] || any_root != (k_root[g] > 0) || (m.b[g] && !any_b))
      return fail(HGNN_E_ARG, "fuse_weights_multi: group %d: outputs / root blocks / biases", g);
    total = std::max<int64_t>(total, (int64_t)h * a.k_tot + (m.b[g] ? h : 0));
  }
  hipLaunchKernelGGL(k_fuse_weights_multi, dim3((unsigned)cdiv(total, 256), (unsigned)n_groups),
                     dim3(256), 0, as_stream(stream), m);
  return check_launch("k_fuse_weights_multi");
}

int hgnn_split_weight_grads_multi(int32_t n_groups, const int32_t* n_rel, const float* const* dw,
                                  const float* const* db, const int32_t* k, const int32_t* k_root,
                                  const float* scale, int32_t h, float* const* dwl,
                                  float* const* dwr, float* const* dbl, hgnn_stream_t stream) {
  if (n_groups < 1 || n_groups > kMaxFuseGroups || !n_rel || !dw || !k || !k_root)
    return fail(HGNN_E_ARG, "split_weight_grads_multi: n_groups=%d (1..%d)", n_groups,
                kMaxFuseGroups);
  FuseMulti m{};
  int64_t total = 1;
  for (int g = 0, base = 0; g < n_groups; base += n_rel[g], ++g) {
    FuseArgs& a = m.g[g];
    if (int rc = fill(a, n_rel[g], k + base, k_root[g], scale + base, h)) return rc;
    if (!dw[g]) return fail(HGNN_E_ARG, "split_weight_grads_multi: dw[%d] is null", g);
    for (int r = 0; r < n_rel[g]; ++r) {
      a.dwl[r] = dwl ? dwl[base + r] : nullptr;
      a.dwr[r] = dwr ? dwr[base + r] : nullptr;
      a.dbl[r] = dbl ? dbl[base + r] : nullptr;
      if (a.dwr[r] && k_root[g] == 0)
        return fail(HGNN_E_ARG, "split_weight_grads_multi: group %d dwr[%d] without a root", g, r);
    }
    m.dw[g] = dw[g];
    m.db[g] = db ? db[g] : nullptr;
    total = std::max<int64_t>(total, (int64_t)h * a.k_tot + (m.db[g] ? h : 0));
  }
  hipLaunchKernelGGL(k_split_weight_grads_multi,
                     dim3((unsigned)cdiv(total, 256), (unsigned)n_groups), dim3(256), 0,
                     as_stream(stream), m);
  return check_launch("k_split_weight_grads_multi");
}

}  // extern "C"
