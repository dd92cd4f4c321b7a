/* hgnn — MI355X (gfx950) hetero message-passing hot path, C ABI.
 *
 * Drop-in boundary for the per-relation SAGE aggregation the reference reaches through PyG
 * (SAGEConv((-1,-1), h) at train_gnn.py:158-160, called at train_gnn.py:177-198,
 * inference.py:143-166, test_gnn.py:141-166).  The reference has no FFI of its own (it is
 * pure Python over torch_geometric), so each entry point below names the PyG/ATen
 * step it replaces; INTEGRATION.md shows the ctypes binding a maintainer adds.
 *
 * Conventions
 *   - every pointer is DEVICE memory owned by the caller (PyTorch's caching allocator in the
 *     shipped host code); the library allocates nothing persistent, scratch comes in `ws`;
 *   - all work is stream-ordered on `stream` (a hipStream_t passed as void*); no host syncs,
 *     no hipMalloc/hipFree inside, so every call can be captured into a hipGraph;
 *   - row-major fp32 feature tables ([rows, d] contiguous); int32 CSR; int64 COO inputs;
 *   - return 0 (HGNN_OK) or an HGNN_E_* code; hgnn_last_error_string() (thread-local) says why.
 */
#ifndef HGNN_H_
#define HGNN_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HGNN_OK 0
#define HGNN_E_ARG 1001         /* bad shape / null pointer / size out of range */
#define HGNN_E_HIP 1002         /* a HIP runtime error (launch failure) */
#define HGNN_E_WS 1003          /* workspace too small */
#define HGNN_E_UNSUPPORTED 1004 /* shape outside what the kernels implement */

#define HGNN_MEAN 1        /* multiply each row sum by 1/deg (deg 0 -> 0) */
#define HGNN_ACCUMULATE 2  /* out += result instead of out = result */

#define HGNN_MAX_SEG 6     /* input segments of one fused linear */

typedef void* hgnn_stream_t; /* hipStream_t */

int hgnn_version(void);
const char* hgnn_last_error_string(void);

/* ---- K5: COO -> CSR, stable (each row keeps the COO edge order) -------------------------------
 * Replaces PyG's implicit scatter over unsorted COO (train_gnn.py:28,55 keep edges chronological;
 * train_gnn.py:128-133 masks out-of-range ids, train_gnn.py:142 flips for rev_engages).
 * Groups edges by key (dst for the forward CSR, src for the backward CSC):
 *   rowptr[n_keys+1], col[e] = other[perm[e]], perm[e] = original edge id.
 * Edges whose key is outside [0,n_keys) or whose other is outside [0,n_other) are dropped (sorted
 * to the end, excluded from rowptr); their count is written to *d_invalid (device int32).
 * E < 2^31.  Workspace: hgnn_coo_to_csr_ws_bytes(E, n_keys). */
size_t hgnn_coo_to_csr_ws_bytes(int64_t E, int64_t n_keys);
int hgnn_coo_to_csr(const int64_t* key, const int64_t* other, int64_t E, int64_t n_keys,
                    int64_t n_other, int32_t* rowptr, int32_t* col, int32_t* perm,
                    int32_t* d_invalid, void* ws, size_t ws_bytes, hgnn_stream_t stream);

/* Stable sort of int32 keys in [0,n_keys) carrying one or two int32 payloads (b may be NULL):
 * rowptr[n_keys+1] over the sorted keys, payloads in key order.  Out-of-range keys are dropped
 * and counted in *d_invalid.  d_invalid == NULL declares the keys already validated (the fused
 * loss validates its negatives in hgnn_edge_score_fwd): no extra pass over the keys then, and an
 * out-of-range key is still never dereferenced, only misplaced.  `keys` is never written.
 * Used per step to group the sampled negatives by post. */
size_t hgnn_sort_pairs_ws_bytes(int64_t E, int64_t n_keys);
int hgnn_sort_pairs_i32(const int32_t* keys, const int32_t* a, const int32_t* b, int64_t E,
                        int64_t n_keys, int32_t* rowptr, int32_t* a_sorted, int32_t* b_sorted,
                        int32_t* d_invalid, void* ws, size_t ws_bytes, hgnn_stream_t stream);

/* As hgnn_sort_pairs_i32 for int64 keys (e.g. torch.randint negatives as drawn): out-of-range
 * keys always go to the dropped sentinel and are counted in *d_invalid (required). */
int hgnn_sort_pairs_i64(const int64_t* keys, const int32_t* a, const int32_t* b, int64_t E,
                        int64_t n_keys, int32_t* rowptr, int32_t* a_sorted, int32_t* b_sorted,
                        int32_t* d_invalid, void* ws, size_t ws_bytes, hgnn_stream_t stream);

/* Transpose of a CSR (rowptr[n_rows+1] / col[E], columns in [0, n_cols) — not re-validated)
 * into its CSC: t_rowptr[n_cols+1], t_col[E] = the row of each entry, t_perm[E] = its CSR
 * position, stable (rows ascending within a column); t_w (nullable) = 1/deg(row) per entry, the
 * weight of the mean's backward.  One call instead of COO -> sort for the backward of a relation
 * whose edges come grouped by destination (sampled blocks).  ws: hgnn_sort_pairs_ws_bytes(E, n_cols). */
int hgnn_csr_transpose(const int32_t* rowptr, const int32_t* col, int64_t n_rows, int64_t E,
                       int64_t n_cols, int32_t* t_rowptr, int32_t* t_col, int32_t* t_perm,
                       float* t_w, void* ws, size_t ws_bytes, hgnn_stream_t stream);

/* hgnn_csr_transpose for n_rel (<= 8) CSRs in one sort (the relations of one sampled block):
 * relation r's CSR rowptr[r][n_rows[r]+1] / col[r][E[r]] with columns in [0, n_cols[r]); outputs
 * per relation exactly as hgnn_csr_transpose's.  ws: hgnn_csr_transpose_multi_ws_bytes(sum of E,
 * sum of n_cols). */
size_t hgnn_csr_transpose_multi_ws_bytes(int64_t E_total, int64_t n_cols_total);
int hgnn_csr_transpose_multi(int32_t n_rel, const int32_t* const* rowptr,
                             const int32_t* const* col, const int64_t* n_rows, const int64_t* E,
                             const int64_t* n_cols, int32_t* const* t_rowptr,
                             int32_t* const* t_col, int32_t* const* t_perm, float* const* t_w,
                             void* ws, size_t ws_bytes, hgnn_stream_t stream);

/* The loss's negatives drawn and grouped in one call: exactly hgnn_uniform_i32(d_seed, E, n_keys,
 * neg_out) followed by hgnn_sort_pairs_i32(neg_out, a, NULL, E, n_keys, rowptr, a_sorted, NULL,
 * NULL, ...), with the draws computed inside the sort's first pass instead of being written and
 * read back (neg_out, E int32 in position order, may be NULL).  Replaces the reference's
 * torch.randint negatives (train_gnn.py:272) plus the grouping the fused dP gather needs.
 * Workspace: hgnn_sort_pairs_ws_bytes(E, n_keys). */
int hgnn_draw_sort_negatives(const uint64_t* d_seed, const int32_t* a, int64_t E, int64_t n_keys,
                             int32_t* neg_out, int32_t* rowptr, int32_t* a_sorted, void* ws,
                             size_t ws_bytes, hgnn_stream_t stream);

/* ---- degree-skew plan ----------------------------------------------------------------------
 * Rows with more than `chunk` edges are split into ceil(deg/chunk) chunks, each summed by its own
 * wave into a partial slot, then reduced in chunk order (deterministic).  Two phases so the host
 * can size the plan: count writes {n_heavy, n_chunks} to d_counts2 (device int32[2]). */
size_t hgnn_plan_ws_bytes(int64_t n_rows);
int hgnn_plan_count(const int32_t* rowptr, int64_t n_rows, int32_t chunk, int32_t* d_counts2,
                    void* ws, size_t ws_bytes, hgnn_stream_t stream);
int hgnn_plan_fill(const int32_t* rowptr, int64_t n_rows, int32_t chunk, int32_t* heavy_rows,
                   int32_t* heavy_first, void* ws, size_t ws_bytes, hgnn_stream_t stream);
/* inv_deg[i] = 1/(rowptr[i+1]-rowptr[i]) or 0 for an empty row. */
int hgnn_inv_degree(const int32_t* rowptr, int64_t n_rows, float* inv_deg, hgnn_stream_t stream);

/* ---- K1/K2: segmented gather-reduce over a CSR ----------------------------------------------
 *   out[i,:] (+)= s_i * sum_{p in [rowptr[i],rowptr[i+1])} w_p * x[col[p],:]
 * with w_p = (edge_w ? edge_w[p] : 1) * (col_w ? col_w[col[p]] : 1), s_i = 1/deg_i under
 * HGNN_MEAN (0 for deg 0), else 1.  Heavy rows follow the plan (slab: n_chunks*d floats).
 * Any d >= 1 (float4 path when d % 4 == 0). */
int hgnn_gather_reduce(const float* x, int64_t n_x, int32_t d, const int32_t* rowptr,
                       const int32_t* col, int64_t n_rows, const float* edge_w,
                       const float* col_w, int32_t flags, const int32_t* heavy_rows,
                       const int32_t* heavy_first, int64_t n_heavy, int64_t n_chunks,
                       int32_t chunk, float* slab, float* out, hgnn_stream_t stream);

/* K1 forward: aggr = mean_{(j->i)} x_src[j]  — PyG propagate(aggr='mean') inside SAGEConv:
 * x_src.index_select(0, src) + scatter(..., dst, reduce='mean'), train_gnn.py:177-198. */
/* n_jobs (<= 8) gathers of one row width in one launch, as hgnn_gather_reduce each (job j: x[j]
 * of n_x[j] rows, rowptr[j] / col[j] over n_rows[j] rows, edge_w[j] nullable, the shared flags)
 * into DISTINCT outputs out[j]; rows are never split (no heavy-row plan: short rows, e.g. sampled
 * blocks), d % 4 == 0 and d <= 512.  With HGNN_ACCUMULATE, acc_limit[j] > 0 (acc_limit nullable)
 * limits the accumulation to rows below it and writes the other rows fresh (a K2 into a gradient
 * whose prefix holds the root term: no zero-fill of the rest).  The per-relation K1s of a sampled
 * layer (and each round of its K2s) as one graph node.  Results exactly those of the single calls
 * (on a zeroed remainder). */
int hgnn_gather_reduce_multi(int32_t n_jobs, const float* const* x, const int64_t* n_x, int32_t d,
                             const int32_t* const* rowptr, const int32_t* const* col,
                             const int64_t* n_rows, const float* const* edge_w, int32_t flags,
                             const int64_t* acc_limit, float* const* out, hgnn_stream_t stream);

/* hgnn_gather_reduce with a per-row output scale: out[i,:] (+)= row_w[i] * sum_p w_p x[col[p],:]
 * (row_w replaces HGNN_MEAN's 1/segment length; not both).  With row_w = 1/deg of the whole
 * relation this is one pass of a mean split over source blocks: the passes over the blocks' CSRs
 * (HGNN_ACCUMULATE from the second on) sum to the relation's mean, each pass reading only its
 * block of the source table. */
int hgnn_gather_reduce_scaled(const float* x, int64_t n_x, int32_t d, const int32_t* rowptr,
                              const int32_t* col, int64_t n_rows, const float* edge_w,
                              const float* col_w, const float* row_w, int32_t flags,
                              const int32_t* heavy_rows, const int32_t* heavy_first,
                              int64_t n_heavy, int64_t n_chunks, int32_t chunk, float* slab,
                              float* out, hgnn_stream_t stream);
int hgnn_gather_mean_fwd(const float* x_src, int64_t n_src, int32_t d, const int32_t* rowptr,
                         const int32_t* col, int64_t n_dst, const int32_t* heavy_rows,
                         const int32_t* heavy_first, int64_t n_heavy, int64_t n_chunks,
                         int32_t chunk, float* slab, float* aggr, hgnn_stream_t stream);

/* K2 backward: grad_x_src[j] (+)= sum_{(j->i)} grad_aggr[i] * inv_deg[i], walking the transposed
 * CSR (grouped by source; t_col holds destinations) — autograd of the mean scatter. */
int hgnn_scatter_mean_bwd(const float* grad_aggr, int64_t n_dst, const float* inv_deg,
                          const int32_t* t_rowptr, const int32_t* t_col, int64_t n_src,
                          int32_t d, const int32_t* heavy_rows, const int32_t* heavy_first,
                          int64_t n_heavy, int64_t n_chunks, int32_t chunk, float* slab,
                          float* grad_x_src, int32_t accumulate, hgnn_stream_t stream);

/* ---- K3/K4: fused multi-segment linear (fp32 MFMA) -------------------------------------------
 * Replaces SAGEConv's lin_l/lin_r addmm plus WeightedRGCN's weighted sum + ReLU
 * (train_gnn.py:187-198):
 *   out[n, h] = act( sum_s xs[s][n, ks[s]] @ w[:, off_s:off_s+ks[s]]^T + bias )
 * w is [h, sum(ks)] row-major (torch Linear layout), act = ReLU when relu != 0.
 * `out` should not alias an input segment: at h = 128 and sum(ks) = 384 / 512 the split kernels
 * run as two column blocks that pass partial rows through `out`, and a call whose `out` overlaps
 * an xs[s] (or `add`) range is routed to the general f32-input kernels instead. */
int hgnn_linear_fwd(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                    const float* w, int32_t h, const float* bias, int32_t relu, float* out,
                    hgnn_stream_t stream);

/* hgnn_linear_fwd with an additive input: out = act( sum_s xs[s] @ w_s^T + bias + add ), add is
 * [n_rows, h] (nullable).  The destination update of a relation whose lin_l was applied to the
 * SOURCE table before the mean gather (mean is linear: lin_l(mean x_j) = mean(lin_l x_j) - 
 * ops.py "pre-projected relations"): add = the gathered projected rows. */
int hgnn_linear_fwd_add(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                        const float* w, int32_t h, const float* bias, const float* add,
                        int32_t relu, float* out, hgnn_stream_t stream);

/* The relation-weighted fused weight of one destination update (WeightedRGCN's
 * relu(w_direct * conv_a + w_social * conv_b), train_gnn.py:187-198, folded into one K3):
 *   w_out = [s_1 wl_1 | ... | s_R wl_R | sum_r s_r wr_r]   ([h, sum_r k_r + k_root], row-major)
 *   b_out = sum_r s_r bl_r                                 (nullable; needs some bl_r)
 * wl[r]: [h, k_r]; wr[r]: [h, k_root] or NULL (no lin_r; k_root = 0 when every wr is NULL);
 * bl[r]: [h] or NULL.  n_rel <= HGNN_MAX_SEG - 1.  Bitwise the torch expression (products and sums
 * rounded separately, in relation order).  Replaces the per-step cat/mul/add chain. */
int hgnn_fuse_weights(int32_t n_rel, const float* const* wl, const int32_t* k,
                      const float* const* wr, int32_t k_root, const float* const* bl,
                      const float* scale, int32_t h, float* w_out, float* b_out,
                      hgnn_stream_t stream);
/* Its adjoint: dwl[r] = s_r dw[:, block r], dwr[r] = s_r dw[:, root block], dbl[r] = s_r db
 * (every output array and entry nullable). */
int hgnn_split_weight_grads(int32_t n_rel, const float* dw, const float* db, const int32_t* k,
                            int32_t k_root, const float* scale, int32_t h, float* const* dwl,
                            float* const* dwr, float* const* dbl, hgnn_stream_t stream);

/* Both for n_groups (<= 4) destination updates of one layer in one launch: group g's relations
 * are the flattened entries [base_g, base_g + n_rel[g]) of wl / k / wr / bl / scale (and of
 * dwl / dwr / dbl), base_g = n_rel[0] + ... + n_rel[g - 1]; w_out[g] / b_out[g] (b_out or its
 * entries nullable) and dw[g] / db[g] per group, h shared.  Results exactly those of the
 * single-update calls. */
int hgnn_fuse_weights_multi(int32_t n_groups, const int32_t* n_rel, const float* const* wl,
                            const int32_t* k, const float* const* wr, const int32_t* k_root,
                            const float* const* bl, const float* scale, int32_t h,
                            float* const* w_out, float* const* b_out, hgnn_stream_t stream);
int hgnn_split_weight_grads_multi(int32_t n_groups, const int32_t* n_rel, const float* const* dw,
                                  const float* const* db, const int32_t* k, const int32_t* k_root,
                                  const float* scale, int32_t h, float* const* dwl,
                                  float* const* dwr, float* const* dbl, hgnn_stream_t stream);

/* hgnn_linear_fwd_add that also writes the ReLU mask of `out` as bits (relu != 0, h % 32 == 0):
 * bit c % 32 of mask[row * (h / 32) + c / 32] = out[row][c] > 0, 16-B aligned.  The backward
 * (hgnn_linear_bwd_mask) reads h/8 bytes per row instead of out's 4h: autograd's saved ReLU
 * output is only ever used for that mask (train_gnn.py:198's activation). */
int hgnn_linear_fwd_mask(int32_t n_seg, const float* const* xs, const int32_t* ks,
                         int64_t n_rows, const float* w, int32_t h, const float* bias,
                         const float* add, int32_t relu, float* out, uint32_t* mask,
                         hgnn_stream_t stream);

/* Backward of hgnn_linear_fwd.  dz = dout * (out > 0) when out != NULL (ReLU), else dout.
 *   dxs[s] = dz @ w[:, seg s]           (skipped for NULL entries)
 *   dw     = dz^T @ [xs...]             (NULL: skipped; same for db = colsum(dz))
 * Deterministic (per-block partials reduced in block order).  Workspace:
 * hgnn_linear_bwd_ws_bytes(n_rows, sum(ks), h). */
size_t hgnn_linear_bwd_ws_bytes(int64_t n_rows, int32_t k_total, int32_t h);
/* hgnn_linear_bwd that also writes the masked dz ([n_rows, h], dz_out) — the gradient a
 * pre-projected relation's K2 scatters (ops.py) — from the pass that masks it anyway. */
int hgnn_linear_bwd_dz(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                       const float* w, int32_t h, const float* dout, const float* out,
                       float* const* dxs, float* dw, float* db, float* dz_out, void* ws,
                       size_t ws_bytes, hgnn_stream_t stream);
/* hgnn_linear_bwd_dz with the ReLU mask also given as the bits of hgnn_linear_fwd_mask: the
 * persistent backward kernels read the bits, the others `out` (both required). */
int hgnn_linear_bwd_mask(int32_t n_seg, const float* const* xs, const int32_t* ks,
                         int64_t n_rows, const float* w, int32_t h, const float* dout,
                         const float* out, const uint32_t* mask, float* const* dxs, float* dw,
                         float* db, float* dz_out, void* ws, size_t ws_bytes,
                         hgnn_stream_t stream);
/* hgnn_linear_bwd_mask where bit s of dx_accumulate adds segment s's input gradient into what
 * dxs[s] already holds instead of storing it: a node table whose gradient has several producers
 * (layer 1's post output at layer 2: the post update's root term and the pre-projected
 * relation's projection) gets the second one in the same pass, not through a separate add —
 * autograd's gradient accumulation of train_gnn.py:283's backward. */
int hgnn_linear_bwd_ex(int32_t n_seg, const float* const* xs, const int32_t* ks,
                       int64_t n_rows, const float* w, int32_t h, const float* dout,
                       const float* out, const uint32_t* mask, float* const* dxs,
                       uint32_t dx_accumulate, float* dw, float* db, float* dz_out, void* ws,
                       size_t ws_bytes, hgnn_stream_t stream);
/* Several K3 calls at once — job j is hgnn_linear_fwd_mask(n_seg[j], the next n_seg[j] entries
 * of xs / ks, n_rows[j], w[j], h, bias[j], NULL, relu[j], out[j], mask[j]) — in one launch per
 * column block where two jobs both take the K = 384 / 512 split path with the same K (a sampled
 * layer's two destination types: ops._HeteroLayer), job by job otherwise.  bias / relu / mask
 * may be NULL (none for every job).  A pair only runs side by side when neither job writes what
 * the other reads (byte ranges checked; else job by job).  Replaces the per-destination-type
 * lin_l / lin_r calls of HeteroConv (reference train_gnn.py:147-200), like hgnn_linear_fwd. */
int hgnn_linear_fwd_multi(int32_t n_jobs, const int32_t* n_seg, const float* const* xs,
                          const int32_t* ks, const int64_t* n_rows, const float* const* w,
                          int32_t h, const float* const* bias, const int32_t* relu,
                          float* const* out, uint32_t* const* mask, hgnn_stream_t stream);
/* Backward of hgnn_linear_fwd_multi: job j is hgnn_linear_bwd_ex(n_seg[j], xs / ks / dxs from
 * the job's entries, n_rows[j], w[j], h, dout[j], out[j], mask[j], dx_accumulate[j], dw[j], db[j],
 * NULL, its workspace).  ws: hgnn_linear_bwd_multi_ws_bytes (the jobs' hgnn_linear_bwd_ws_bytes
 * one after the other).  out / mask / dx_accumulate / dw / db may be NULL (none for every job). */
size_t hgnn_linear_bwd_multi_ws_bytes(int32_t n_jobs, const int64_t* n_rows,
                                      const int32_t* k_total, int32_t h);
int hgnn_linear_bwd_multi(int32_t n_jobs, const int32_t* n_seg, const float* const* xs,
                          const int32_t* ks, const int64_t* n_rows, const float* const* w,
                          int32_t h, const float* const* dout, const float* const* out,
                          const uint32_t* const* mask, float* const* dxs,
                          const uint32_t* dx_accumulate, float* const* dw, float* const* db,
                          void* ws, size_t ws_bytes, hgnn_stream_t stream);
/* Adam (torch.optim.Adam, the reference's optimizer: train_gnn.py:207) over n_tensors fp32
 * parameters in one launch (per 32 tensors): p, m, v updated in place from g.  step: one device
 * float, the steps done so far — the launch uses step + 1 and writes it back once every block has
 * read it (capturable: no host value); done: one device uint32, zero between launches (the
 * launch leaves it zero).  One update per (step, done) pair in flight. */
int hgnn_adam_multi(int32_t n_tensors, float* const* params, const float* const* grads,
                    float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                    float* step, uint32_t* done, double lr, double beta1, double beta2, double eps,
                    double weight_decay, hgnn_stream_t stream);
int hgnn_linear_bwd(int32_t n_seg, const float* const* xs, const int32_t* ks, int64_t n_rows,
                    const float* w, int32_t h, const float* dout, const float* out,
                    float* const* dxs, float* dw, float* db, void* ws, size_t ws_bytes,
                    hgnn_stream_t stream);

/* dP of the fused loss with each edge's weight recomputed from its score (no weight arrays):
 *   out[r,:] (+)= sum_{p in row r} w(<x[col[p]],:>, rowvec[r,:]>) * x[col[p],:]
 *   mode 1 (positive edges): w(s) = c*inv_e*(sigmoid(s) - 1), c = *cscale
 *   mode 2 (negative edges): w(s) = inv_e*sigmoid(s)
 * i.e. dL/dP[r] of hgnn_edge_score_fwd's loss (train_gnn.py:276-281) for x = U, rowvec = P.
 * Heavy rows / slab as hgnn_gather_reduce. */
int hgnn_score_gather(const float* x, int64_t n_x, const float* rowvec, int32_t d,
                      const int32_t* rowptr, const int32_t* col, int64_t n_rows, int32_t mode,
                      const float* cscale, float inv_e, const int32_t* heavy_rows,
                      const int32_t* heavy_first, int64_t n_heavy, int64_t n_chunks,
                      int32_t chunk, float* slab, float* out, int32_t accumulate,
                      hgnn_stream_t stream);

/* Both dP gathers of the fused loss in one pass (replaces a mode-1 hgnn_score_gather over the
 * positives followed by an accumulating mode-2 one over the negatives):
 *   out[r,:] = sum_{p in rowptr/col row r} w_1(s) x[col[p],:]  +  sum_{p in rowptr_n/col_n row r}
 *              w_2(s) x[col_n[p],:]
 * with w_1, w_2 as hgnn_score_gather's modes 1 and 2.  The heavy-row plan applies to the positive
 * list only (the uniform negatives have no heavy rows); every row is written (no accumulate). */
int hgnn_score_gather2(const float* x, int64_t n_x, const float* rowvec, int32_t d,
                       const int32_t* rowptr, const int32_t* col, const int32_t* rowptr_n,
                       const int32_t* col_n, int64_t n_rows, const float* cscale, float inv_e,
                       const int32_t* heavy_rows, const int32_t* heavy_first, int64_t n_heavy,
                       int64_t n_chunks, int32_t chunk, float* slab, float* out,
                       hgnn_stream_t stream);

/* ---- edge scoring + weighted BCE (train_gnn.py:259-281), fused with its gradient --------------
 * Positive edges grouped by user (rowptr_u/col_u = post ids); neg_u_order[k] = the negative post
 * drawn for position k; to_post_pos[k] = that edge's position in the post-grouped CSR.
 *   loss = c * mean softplus(-<U[u],P[p]>) + mean softplus(<U[u],P[n]>),  c = *cscale
 *          (= mean(pos_weights): BCEWithLogitsLoss() reduces to a scalar first)
 * Writes dU (dL/dU for a unit upstream gradient, row-owned, no atomics).  Optional (may be NULL):
 * per position (neg_key, neg_user) — the validated negative and its user, for sorting by post;
 * hpos[post-grouped
 * pos] (weight of U[u] in dP[p], needs to_post_pos) and neg_w (weight in dP[n]) — not needed when
 * dP is formed by hgnn_score_gather, which recomputes both;
 * part needs hgnn_edge_score_parts(n_users) floats (16-B aligned); *err counts out-of-range negatives
 * (err nullable: not counted — a caller whose negatives are valid by construction). */
int64_t hgnn_edge_score_parts(int64_t n_users);
int hgnn_edge_score_fwd(const float* U, const float* P, int32_t d, int64_t n_users,
                        int64_t n_posts, const int32_t* rowptr_u, const int32_t* col_u,
                        const int64_t* neg_u_order, const int32_t* to_post_pos, int64_t n_edges,
                        const float* cscale, float* dU, float* hpos, int32_t* neg_key,
                        int32_t* neg_user, float* neg_w, float* part, float* loss, int32_t* err,
                        hgnn_stream_t stream);

/* K3 at H = 128 and K = 128 / 256 runs on bf16 MFMA as an fp32-exact three-piece split (each
 * fp32 operand = three bf16 pieces, six piece products per fp32 product, f32 accumulation:
 * fp32-class error; each operand element split once per block), and K = 384 / 512
 * (every segment a multiple of 16 columns) as two column blocks on the same kernels, unless
 * HGNN_K3_X6=0.  on = 1 / 0 selects the split or the f32-input MFMA kernels for the calls that
 * follow (process-wide, not thread-safe against calls in flight); on < 0 only queries.  Returns
 * the previous setting. */
int hgnn_set_k3_split(int32_t on);

/* Single-input forms, one PyG Linear at a time (SURVEY §8b names; same kernels as above):
 *   hgnn_linear_fwd_f32:   out[n,h] = x[n,k] @ w[h,k]^T (+ bias[h] when non-NULL)
 *   hgnn_linear_dgrad_f32: dx[n,k]  = dy[n,h] @ w
 *   hgnn_linear_wgrad_f32: dw[h,k]  = dy^T @ x, db[h] = colsum(dy) (db may be NULL);
 *                          ws: hgnn_linear_bwd_ws_bytes(n, k, h) */
int hgnn_linear_fwd_f32(const float* x, int64_t n_rows, int32_t k, const float* w, int32_t h,
                        const float* bias, float* out, hgnn_stream_t stream);
int hgnn_linear_dgrad_f32(const float* dy, int64_t n_rows, int32_t h, const float* w, int32_t k,
                          float* dx, hgnn_stream_t stream);
int hgnn_linear_wgrad_f32(const float* x, const float* dy, int64_t n_rows, int32_t k, int32_t h,
                          float* dw, float* db, void* ws, size_t ws_bytes, hgnn_stream_t stream);

/* ---- K4 standalone: WeightedRGCN's weighted relation sum + ReLU (train_gnn.py:187-198) -------
 *   out[e] = act( sum_r weights[r] * ins[r][e] ),  e < n elements, n_in <= HGNN_MAX_SEG
 * (weights: HOST array; ins: HOST array of device pointers).  The model path folds this into K3;
 * these are for callers that combine per-relation SAGEConv outputs themselves.
 * Backward: dins[r][e] = weights[r] * dout[e] * (relu ? out[e] > 0 : 1)  (NULL dins[r] skipped). */
int hgnn_hetero_epilogue(int32_t n_in, const float* const* ins, const float* weights, int64_t n,
                         int32_t relu, float* out, hgnn_stream_t stream);
int hgnn_hetero_epilogue_bwd(int32_t n_in, const float* weights, int64_t n, int32_t relu,
                             const float* out, const float* dout, float* const* dins,
                             hgnn_stream_t stream);

/* hgnn_edge_score_fwd with int32 negatives (as hgnn_uniform_i32 draws them) and without the
 * optional per-position outputs (the dP side is formed by hgnn_score_gather). */
int hgnn_edge_score_fwd_i32(const float* U, const float* P, int32_t d, int64_t n_users,
                            int64_t n_posts, const int32_t* rowptr_u, const int32_t* col_u,
                            const int32_t* neg_u_order, int64_t n_edges, const float* cscale,
                            float* dU, float* part, float* loss, int32_t* err,
                            hgnn_stream_t stream);
/* hgnn_edge_score_fwd_i32 with the negatives drawn in the kernel: the negative of position k is
 * the draw hgnn_uniform_i32(d_seed, n_edges, n_posts) would write at k (train_gnn.py:272's
 * torch.randint, one per positive edge), so no position-order array is written or read (the
 * fused loss passes neg_out = NULL to hgnn_draw_sort_negatives and this the same seed). */
int hgnn_edge_score_fwd_draw(const float* U, const float* P, int32_t d, int64_t n_users,
                             int64_t n_posts, const int32_t* rowptr_u, const int32_t* col_u,
                             const uint64_t* d_seed, int64_t n_edges, const float* cscale,
                             float* dU, float* part, float* loss, int32_t* err,
                             hgnn_stream_t stream);
/* n uniform int32 draws in [0, hi) (the negatives of train_gnn.py:272), counter-based from the
 * 64-bit seed at d_seed (device memory: a torch Generator draws it without a host sync). */
int hgnn_uniform_i32(const uint64_t* d_seed, int64_t n, int32_t hi, int32_t* out,
                     hgnn_stream_t stream);
/* x[0:n] *= *d_scale in place, a no-op when *d_scale == 1 (read on the device).  The fused
 * loss's autograd backward: its dU/dP are formed in the forward and scaled by the incoming
 * gradient (1 for loss.backward()).  x 16-byte aligned. */
int hgnn_scale_unless_one(float* x, int64_t n, const float* d_scale, hgnn_stream_t stream);

/* ---- neighbour sampling for mini-batches (BASELINE cfg5; no reference counterpart) -----------
 * For each destination dst_ids[i] (rows of a destination-grouped CSR rowptr/col over n_rows):
 * keep all in-neighbours if deg <= fanout (or fanout < 0), else `fanout` distinct neighbour
 * positions drawn uniformly (Floyd's algorithm, counter-based hash of (seed, dst id, draw)).
 * out_rowptr[n_dst+1] is written first; with out_col == NULL only the counts are produced (read
 * out_rowptr[n_dst] to size out_col).  fanout in 1..64 or < 0.  ws: hgnn_sample_ws_bytes(n_dst). */
size_t hgnn_sample_ws_bytes(int64_t n_dst);
int hgnn_sample_neighbors(const int32_t* rowptr, const int32_t* col, int64_t n_rows,
                          const int32_t* dst_ids, int64_t n_dst, int32_t fanout, uint64_t seed,
                          int32_t* out_rowptr, int32_t* out_col, void* ws, size_t ws_bytes,
                          hgnn_stream_t stream);
/* The fill phase alone, for an out_rowptr an earlier count-only hgnn_sample_neighbors call made
 * (same rowptr, dst_ids, fanout): one launch.  Destination ids outside [0, n_rows) have no
 * neighbours in either phase (never dereferenced). */
int hgnn_sample_fill(const int32_t* rowptr, const int32_t* col, int64_t n_rows,
                     const int32_t* dst_ids, int64_t n_dst, int32_t fanout, uint64_t seed,
                     const int32_t* out_rowptr, int32_t* out_col, hgnn_stream_t stream);
/* One hop of the sampler over every relation into the frontier (at most 8), one launch per phase
 * (hgnn_sample_neighbors / hgnn_sample_fill per relation, batched; the samples are identical).
 * Count: out_rowptrs[r][n_dst[r]+1] zero-based per relation, d_totals[r] (device int32) = its
 * size; ws: hgnn_sample_hop_ws_bytes(sum of n_dst).  Fill: relation r's sample into out_cols[r]
 * (d_totals[r] entries).  Host arrays of n_rel entries; one fanout and seed for the hop. */
size_t hgnn_sample_hop_ws_bytes(int64_t n_total_dst);
int hgnn_sample_hop_count(int32_t n_rel, const int32_t* const* rowptrs, const int64_t* n_rows,
                          const int32_t* const* dst_ids, const int64_t* n_dst, int32_t fanout,
                          int32_t* const* out_rowptrs, int32_t* d_totals, void* ws,
                          size_t ws_bytes, hgnn_stream_t stream);
int hgnn_sample_hop_fill(int32_t n_rel, const int32_t* const* rowptrs, const int32_t* const* cols,
                         const int64_t* n_rows, const int32_t* const* dst_ids,
                         const int64_t* n_dst, int32_t fanout, uint64_t seed,
                         const int32_t* const* out_rowptrs, int32_t* const* out_cols,
                         hgnn_stream_t stream);

/* Next layer's node set of one type: nodes_out = [prefix (order kept), then every item id not in
 * prefix, once, in order of first appearance in items]; local_out[k] = position of items[k] in
 * nodes_out; *d_count = total.  Prefix ids distinct; ids are non-negative int32.  nodes_out holds
 * n_prefix + n_items entries.  O(n_prefix + n_items) work (a hash set over this call's ids),
 * deterministic.  ws: hgnn_relabel_ws_bytes(n_prefix, n_items). */
size_t hgnn_relabel_ws_bytes(int64_t n_prefix, int64_t n_items);
int hgnn_relabel(const int32_t* prefix, int64_t n_prefix, const int32_t* items, int64_t n_items,
                 int32_t* local_out, int32_t* nodes_out, int32_t* d_count, void* ws,
                 size_t ws_bytes, hgnn_stream_t stream);
/* hgnn_relabel that also checks the prefix (a mini-batch's seeds): d_count2[0] = the count,
 * d_count2[1] = flags, bit 0 a repeated prefix id, bit 1 a prefix id outside [0, id_limit)
 * (id_limit 0: a type with no nodes, every id flagged; id_limit < 0: no range check).
 * The outputs are unspecified when a flag is set; nothing is read out of bounds. */
int hgnn_relabel_checked(const int32_t* prefix, int64_t n_prefix, int64_t id_limit,
                         const int32_t* items, int64_t n_items, int32_t* local_out,
                         int32_t* nodes_out, int32_t* d_count2, void* ws, size_t ws_bytes,
                         hgnn_stream_t stream);
/* Every node type of a hop in one call (n_types <= 8): type t's prefix prefix[t][n_prefix[t]],
 * its items the consecutive range n_items[t] of `items` (types in order), its node set into
 * nodes_out[t] (n_prefix[t] + n_items[t] entries), the local ids of all items into local_out
 * (per type, as hgnn_relabel); ids < id_limit[t] (required when n_types > 1: the table is keyed
 * by id * n_types + t, so id_limit * n_types < 2^31).  d_count2: with check, (count, flags) per
 * type as hgnn_relabel_checked; without, the counts only.  The same nodes and local ids as one
 * hgnn_relabel per type.  ws: hgnn_relabel_multi_ws_bytes(sum of n_prefix, sum of n_items). */
size_t hgnn_relabel_multi_ws_bytes(int64_t n_prefix_total, int64_t n_items_total);
int hgnn_relabel_multi(int32_t n_types, const int32_t* const* prefix, const int64_t* n_prefix,
                       const int64_t* id_limit, const int32_t* items, const int64_t* n_items,
                       int32_t* local_out, int32_t* const* nodes_out, int32_t* d_count2,
                       int32_t check, void* ws, size_t ws_bytes, hgnn_stream_t stream);

/* Static-capacity copies of sampled blocks (a captured mini-batch step replays one HIP graph over
 * fixed buffers).  Item i (n_items <= 16): the CSR rowptr[i] (n_dst[i] + 1) / col[i] (e[i]) into
 * rowptr_out[i] (d_cap[i] + 1) / col_out[i] (e_cap[i]); the e_cap - e padding entries get sources
 * dummy[i] + (k mod spread[i]) (spread optional, >= 1: padded source rows taken in turn, so the
 * transposed grouping has no long row) and are spread over the padded rows n_dst .. d_cap - 1
 * (d_cap > n_dst required when
 * e_cap > e), so the copy is a valid CSR of d_cap rows whose first n_dst rows are the input's.
 * map[i] (optional): real entries become map[i][col] (a block's local ids -> global ids).
 * d_cap[i] < 0: col only (a node-id list padded with dummy[i]).  Replaces nothing in the
 * reference (which trains full-batch); it feeds forward_blocks' static form (minibatch.py). */
int hgnn_pad_csr_multi(int32_t n_items, const int32_t* const* rowptr, const int32_t* const* col,
                       const int32_t* const* map, const int64_t* n_dst, const int64_t* e,
                       int32_t* const* rowptr_out, int32_t* const* col_out, const int64_t* d_cap,
                       const int64_t* e_cap, const int32_t* dummy, const int32_t* spread,
                       hgnn_stream_t stream);

/* The outermost block's destination rows of a static step (minibatch.StaticBlocks.prepare),
 * gathered with the staged batch in one launch: item i (n_items <= 8) writes
 * out[i][r][0..d) = src[i][ids[i][r]][0..d) for r < n_rows[i]; d % 4 == 0, 16-byte aligned rows,
 * ids in range (not validated).  Replaces the per-type x.index_select of the captured step. */
int hgnn_gather_rows_multi(int32_t n_items, const float* const* src, const int32_t* const* ids,
                           const int64_t* n_rows, int64_t d, float* const* out,
                           hgnn_stream_t stream);

/* A link mini-batch's loss structures in one call (minibatch.LinkLoss.prepare; the reference's
 * loss, train_gnn.py:259-281, over a batch's positive pairs and their negatives): the E pairs
 * (pu[i], pp[i]) with negative pn[i] — local ids, users < n_users, posts < n_posts, not
 * validated — grouped by user, stable: rowptr_u[n_users+1], col_p / neg / uop[E] (post, negative,
 * user per position); the same pairs by post (hgnn_csr_transpose of rowptr_u / col_p: p_rowptr
 * [n_posts+1], p_users / p_perm[E]); the negatives by post (hgnn_sort_pairs_i32(neg, uop):
 * n_rowptr[n_posts+1], n_users_sorted[E]) — the dP gather's order.  Exactly the three calls it
 * replaces.  ws: hgnn_link_group_ws_bytes(E). */
size_t hgnn_link_group_ws_bytes(int64_t E);
int hgnn_link_group(const int32_t* pu, const int32_t* pp, const int32_t* pn, int64_t E,
                    int64_t n_users, int64_t n_posts, int32_t* rowptr_u, int32_t* col_p,
                    int32_t* neg, int32_t* uop, int32_t* p_rowptr, int32_t* p_users,
                    int32_t* p_perm, int32_t* n_rowptr, int32_t* n_users_sorted, void* ws,
                    size_t ws_bytes, hgnn_stream_t stream);

/* ---- sync-free static sampling (minibatch.StaticSampler; csrc/sampler_static.hip) ------------
 * The eager sampler's results (hgnn_sample_hop_count / _fill, hgnn_relabel_multi) followed by
 * hgnn_pad_csr_multi, written straight into static-capacity buffers with every count kept on
 * the device, so a batch is queued without a host read-back.  Not in the reference (it trains
 * full-batch, train_gnn.py:254); it feeds the captured cfg5 step.
 *
 * hgnn_link_seeds: a link batch (minibatch.link_batch): the B <= 2048 positives edge_ids into the
 * (src, dst) rows of the positive relation and their negatives neg[B] (int64 ids < 2^31 - 1);
 * seeds_u[B] / seeds_p[2B] = the distinct users / posts (positives' posts and negatives)
 * ascending, d_counts[2] = their numbers, pu / pp / pn[B] = each pair's local ids (ranks). */
int hgnn_link_seeds(const int64_t* src, const int64_t* dst, const int64_t* edge_ids,
                    const int64_t* neg, int64_t B, int32_t* seeds_u, int32_t* seeds_p,
                    int32_t* pu, int32_t* pp, int32_t* pn, int32_t* d_counts,
                    hgnn_stream_t stream);

/* One hop of n_rel (<= 8) relations, fanout 1..64: relation r samples the first *d_n_dst[r] ids
 * of dst_ids[r] (global CSR rowptrs[r] / cols[r] over n_rows[r] destinations; the count lives on
 * the device, caps[r] bounds it and leaves >= 1 padded row) exactly as hgnn_sample_hop_fill with
 * `seed`: out_rowptrs[r][caps[r] + 1] = the real rows then padded rows spread as
 * hgnn_pad_csr_multi does, fill_outs[r] = the sampled global source ids in CSR order,
 * tail_outs[r][E .. ecaps[r]) = padding entries dummy[r] + (k mod spread[r]), d_E[r] = E.
 * ws: hgnn_sample_hop_ws_bytes(sum of caps). */
int hgnn_sample_hop_static(int32_t n_rel, const int32_t* const* rowptrs,
                           const int32_t* const* cols, const int64_t* n_rows,
                           const int32_t* const* dst_ids, const int32_t* const* d_n_dst,
                           const int64_t* caps, const int64_t* ecaps, int32_t fanout,
                           uint64_t seed, int32_t* const* out_rowptrs, int32_t* const* fill_outs,
                           int32_t* const* tail_outs, const int32_t* dummy,
                           const int32_t* spread, int32_t* d_E, void* ws, size_t ws_bytes,
                           hgnn_stream_t stream);

/* hgnn_relabel_multi over capacity layouts: type ty's prefix = the first *d_n_prefix[ty] ids of
 * prefix[ty]; the items are n_irel (<= 8) relations' runs, relation q in slots item_caps[q] long
 * (consecutive, grouped by source type irel_type[q] ascending), its first d_E[q] valid.  Writes
 * nodes_out[ty] (zeroed past the count up to nodes_caps[ty]), each valid item's local id into
 * local_out[q], d_count[ty] = the node counts.  ws: hgnn_relabel_static_ws_bytes(sum of
 * prefix_caps, sum of item_caps). */
size_t hgnn_relabel_static_ws_bytes(int64_t prefix_cap_total, int64_t item_cap_total);
int hgnn_relabel_static(int32_t n_types, const int32_t* const* prefix,
                        const int32_t* const* d_n_prefix, const int64_t* prefix_caps,
                        int32_t* const* nodes_out, const int64_t* nodes_caps, int32_t n_irel,
                        const int32_t* items, const int64_t* item_caps, const int32_t* irel_type,
                        const int32_t* d_E, int32_t* const* local_out, int32_t* d_count,
                        void* ws, size_t ws_bytes, hgnn_stream_t stream);

/* ---- ranking metrics of the evaluation (train_gnn.py:289-367), batched ----------------------
 * scores [n_rows][ld]: one row per test user over the n_cand sorted test candidates (a GEMM of
 * user and candidate embeddings, computed by the caller).  Per row:
 *   top-k, k = min(K, n_cand), ordered by (score desc, candidate index asc)  -> topk_idx (opt.)
 *   recall[r] = |top-k ∩ true(r)| / true_count[r]   (true_count counts duplicate test edges)
 *   ndcg[r]   = sklearn ndcg_score(binary relevance, scores, k=K), tie-averaged (ignore_ties=False)
 * true_rowptr/true_cand: each row's sorted unique relevant candidate indices.  K <= 63.
 * Scores are assumed finite. */
int hgnn_topk_metrics(const float* scores, int64_t n_rows, int64_t n_cand, int64_t ld,
                      const int32_t* true_rowptr, const int32_t* true_cand,
                      const int32_t* true_count, int32_t K, int32_t* topk_idx, double* recall,
                      double* ndcg, hgnn_stream_t stream);

/* ---- edge construction from raw ids -------------------------------------------
 * Replaces the host loops that map entity ids to node indices row by row:
 * build_edge_index_safe (train_gnn.py:40-73), build_test_edges (test_gnn.py:34-55) and the
 * Series.map(dict) + dropna of build_graph.py:383-402.
 *
 * An id map is a dict {key: value} as an open-addressing table of 16-B slots in device memory.
 * Keys are integers (key_ints[n]) or strings in the Arrow layout (key_offsets[n+1] int64 byte
 * offsets into key_bytes, UTF-8; key_bytes and q_bytes must be readable 16 bytes past their last
 * string, as Arrow's 64-B buffer padding guarantees); keys distinct.  capacity: hgnn_idmap_capacity(n_keys) (a power
 * of two >= 2 n_keys, >= 16); slots: 16·capacity bytes.  The key arrays (and vals) must stay alive
 * for lookups: the table stores key rows, and string matches are confirmed byte by byte. */
int64_t hgnn_idmap_capacity(int64_t n_keys);
int hgnn_idmap_build(const int64_t* key_ints, const int64_t* key_offsets, const uint8_t* key_bytes,
                     int64_t n_keys, void* slots, int64_t capacity, hgnn_stream_t stream);
/* dict.get for n_q queries: out[q] = vals[row of the key equal to query q], or -1 when absent or
 * q_valid[q] == 0 (q_valid may be NULL).  vals == NULL returns the key row.  Integer queries
 * (q_ints) need an integer-keyed map; string queries (q_offsets + q_bytes) a string-keyed one. */
int hgnn_idmap_lookup(const void* slots, int64_t capacity, const int64_t* key_ints,
                      const int64_t* key_offsets, const uint8_t* key_bytes, const int64_t* vals,
                      const int64_t* q_ints, const int64_t* q_offsets, const uint8_t* q_bytes,
                      const uint8_t* q_valid, int64_t n_q, int64_t* out, hgnn_stream_t stream);
/* Keep the rows i in [0,n) whose every column cols[c][i] >= 0 (c < n_cols <= 4), in order:
 * outs[o][k] = cols[out_col[o]][i] for the k-th kept row (n_outs <= 4; one column may feed several
 * outputs, e.g. the post column of both the engage and the author edge list).  *d_count (device)
 * = kept rows; with n_outs == 0 only the count is produced.  n < 2^31.
 * ws: hgnn_compact_rows_ws_bytes(n).  cols/outs/out_col are HOST arrays of device pointers. */
size_t hgnn_compact_rows_ws_bytes(int64_t n);
int hgnn_compact_rows(const int64_t* const* cols, int32_t n_cols, int64_t n,
                      int64_t* const* outs, const int32_t* out_col, int32_t n_outs,
                      int32_t* d_count, void* ws, size_t ws_bytes, hgnn_stream_t stream);

/* As hgnn_topk_metrics for a subset of rows: score row r belongs to row row_map[r] of the true
 * sets and of recall / ndcg (topk_idx stays indexed by r). */
int hgnn_topk_metrics_rows(const float* scores, int64_t n_rows, int64_t n_cand, int64_t ld,
                           const int32_t* row_map, const int32_t* true_rowptr,
                           const int32_t* true_cand, const int32_t* true_count, int32_t K,
                           int32_t* topk_idx, double* recall, double* ndcg, hgnn_stream_t stream);

/* Fused scoring + top-L (the evaluation's GEMM and torch.topk, train_gnn.py:330-340, and
 * inference.py:427-429): for each output row r (user U[rows ? rows[r] : r], d floats) the L best
 * of the n_cand candidates P[c] by <U, P[c]> (fp32 MFMA), score desc then index asc, written to
 * topv / topi [n_rows][L].  The [rows, n_cand] score matrix is never materialised.
 * d in {64, 128}; U and P row-major, 16-B aligned; 1 <= L <= min(64, n_cand). */
size_t hgnn_score_topk_lds_bytes(int32_t d, int32_t L);
int hgnn_score_topk(const float* U, const int32_t* rows, int64_t n_rows, const float* P,
                    int64_t n_cand, int32_t d, int32_t L, float* topv, int32_t* topi,
                    hgnn_stream_t stream);
/* Recall / NDCG (as hgnn_topk_metrics) from hgnn_score_topk lists with L = min(K, n_cand) + 1
 * (or min(K, n_cand) when n_cand <= K).  A row whose K-th value ties the (K+1)-th needs the whole
 * row for sklearn's tie groups: it gets tie_flag = 1 and no outputs; redo those rows with
 * materialised scores (hgnn_topk_metrics_rows). */
int hgnn_topk_finish(const float* topv, const int32_t* topi, int64_t n_rows, int32_t L,
                     int64_t n_cand, int32_t K, const int32_t* true_rowptr,
                     const int32_t* true_cand, const int32_t* true_count, double* recall,
                     double* ndcg, int32_t* tie_flag, hgnn_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* HGNN_H_ */
