"""Batched Recall@K / NDCG@K — the reference's ``evaluate`` (train_gnn.py:289-367) on device.

The reference loops over test users in Python: one [1,d]x[d,C] product, one ``torch.topk``, one
``sklearn.metrics.ndcg_score`` and several host syncs per user.  Here the grouping is a handful of
device sorts; then, for d in (64, 128), one fused kernel scores every test user against every
candidate on MFMA and keeps each user's top-(K+1) list without materialising the scores
(``hgnn_score_topk``), and a second one turns the lists into Recall/NDCG (``hgnn_topk_finish``).
The rare rows whose K-th score ties the next (sklearn's tie groups then need the whole row) and
other widths take the materialised path: one GEMM per user batch (torch.mm -> hipBLASLt) and
``hgnn_topk_metrics`` over it.  Same arguments, same return values.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from . import _native as N


class _Grouped:
    """Test edges grouped per user: candidates, per-user unique relevant candidates, counts."""

    def __init__(self, test_edges: torch.Tensor, num_users: int, num_posts: int):
        te = test_edges.to(torch.int64)
        u, p_local = te[0], te[1] - num_users             # train_gnn.py:313-316
        if p_local.numel() and (int(p_local.min()) < 0 or int(p_local.max()) >= num_posts):
            raise ValueError("evaluate: test edge post id outside [num_users, num_users+num_posts)")
        if u.numel() and int(u.min()) < 0:
            raise ValueError("evaluate: negative user id in test_edges")
        # candidates: every post of the test set, sorted (train_gnn.py:320-322) — including the
        # posts of skipped (out-of-range) users, as in the reference
        self.cand, inv = torch.unique(p_local, sorted=True, return_inverse=True)
        C = int(self.cand.numel())
        keep = u < num_users                              # train_gnn.py:328
        u, c = u[keep], inv[keep]
        self.users, counts = torch.unique(u, sorted=True, return_counts=True)
        self.true_count = counts.to(torch.int32)
        key = torch.unique(u * max(C, 1) + c, sorted=True)     # (user, candidate) pairs, deduped
        ku = key // max(C, 1)
        per_user = torch.searchsorted(ku, self.users, right=True)
        self.rowptr = torch.cat([per_user.new_zeros(1), per_user]).to(torch.int32)
        self.true_cand = (key % max(C, 1)).to(torch.int32)


def _fused_ok(d: int, fused: Optional[bool]) -> bool:
    if fused is None:
        return d in (64, 128)
    if fused and d not in (64, 128):
        raise ValueError(f"fused scoring supports d in (64, 128), got {d}")
    return fused


def evaluate(test_edges: torch.Tensor, user_emb: torch.Tensor, post_emb: torch.Tensor,
             K: int = 10, num_users: Optional[int] = None,
             batch_scores: int = 1 << 30, fused: Optional[bool] = None) -> Tuple[float, float]:
    """Mean Recall@K and NDCG@K over the test users (train_gnn.py:289-367).

    ``test_edges``: [2, E] user -> global post id (post ids offset by ``num_users``, as the
    reference builds them; ``num_users`` defaults to ``user_emb.shape[0]``, the reference's global).
    ``batch_scores`` bounds the floats of one materialised score matrix (rows x candidates).
    ``fused`` (default: when d is 64 or 128) scores and ranks in one kernel without materialising
    the scores (hgnn_score_topk); rows whose K-th score ties the next one are redone on the
    materialised path, which sklearn's tie groups need."""
    dev = N.require_device(user_emb, post_emb, test_edges)
    if user_emb.dtype != torch.float32 or post_emb.dtype != torch.float32:
        raise TypeError("evaluate: fp32 embeddings expected (the reference dtype)")
    nu = int(user_emb.shape[0]) if num_users is None else int(num_users)
    g = _Grouped(test_edges, nu, int(post_emb.shape[0]))
    n_rows, C = int(g.users.numel()), int(g.cand.numel())
    if n_rows == 0:
        return math.nan, math.nan                         # np.mean([]) in the reference
    d = int(user_emb.shape[1])
    ld = (C + 3) // 4 * 4                                  # 16-B aligned score rows
    P_c = post_emb.new_zeros(ld, d)                        # candidates, zero-padded to ld
    P_c[:C] = post_emb.index_select(0, g.cand)
    recall = torch.empty(n_rows, dtype=torch.float64, device=dev)
    ndcg = torch.empty(n_rows, dtype=torch.float64, device=dev)
    lib = N.lib()
    users32 = g.users.to(torch.int32)
    if _fused_ok(d, fused):
        k = min(K, C)
        L = k + 1 if C > k else k
        U = user_emb.contiguous()
        topv = torch.empty(n_rows, L, dtype=torch.float32, device=dev)
        topi = torch.empty(n_rows, L, dtype=torch.int32, device=dev)
        tie = torch.empty(n_rows, dtype=torch.int32, device=dev)
        N.check(lib.hgnn_score_topk(N.ptr(U), N.ptr(users32), n_rows, N.ptr(P_c), C, d, L,
                                    N.ptr(topv), N.ptr(topi), N.stream_ptr(dev)),
                "hgnn_score_topk")
        N.check(lib.hgnn_topk_finish(N.ptr(topv), N.ptr(topi), n_rows, L, C, K, N.ptr(g.rowptr),
                                     N.ptr(g.true_cand), N.ptr(g.true_count), N.ptr(recall),
                                     N.ptr(ndcg), N.ptr(tie), N.stream_ptr(dev)),
                "hgnn_topk_finish")
        redo = torch.nonzero(tie).reshape(-1).to(torch.int32)   # one sync
        n_redo = int(redo.numel())
    else:
        redo, n_redo = None, n_rows                        # every row on the materialised path
    if n_redo:
        rows = max(1, min(n_redo, batch_scores // ld))
        buf = torch.empty(rows, ld, dtype=torch.float32, device=dev)
        for r0 in range(0, n_redo, rows):
            r1 = min(n_redo, r0 + rows)
            S = buf[: r1 - r0]                             # columns >= C (padding) are ignored
            rmap = (torch.arange(r0, r1, dtype=torch.int32, device=dev) if redo is None
                    else redo[r0:r1])
            torch.mm(user_emb.index_select(0, users32[rmap.long()]), P_c.T, out=S)
            N.check(lib.hgnn_topk_metrics_rows(
                N.ptr(S), r1 - r0, C, ld, N.ptr(rmap), N.ptr(g.rowptr), N.ptr(g.true_cand),
                N.ptr(g.true_count), K, None, N.ptr(recall), N.ptr(ndcg), N.stream_ptr(dev)),
                "hgnn_topk_metrics_rows")
    return float(recall.mean()), float(ndcg.mean())


def topk_metrics(scores: torch.Tensor, true_rowptr: torch.Tensor, true_cand: torch.Tensor,
                 true_count: torch.Tensor, K: int = 10):
    """Raw kernel: per-row (topk_idx, recall, ndcg) of a [rows, C] score matrix."""
    dev = N.require_device(scores, true_rowptr, true_cand, true_count)
    n, C = scores.shape
    k = min(K, C)
    topk = torch.empty(n, k, dtype=torch.int32, device=dev)
    recall = torch.empty(n, dtype=torch.float64, device=dev)
    ndcg = torch.empty(n, dtype=torch.float64, device=dev)
    N.check(N.lib().hgnn_topk_metrics(
        N.ptr(scores), n, C, scores.stride(0), N.ptr(true_rowptr), N.ptr(true_cand),
        N.ptr(true_count), K, N.ptr(topk), N.ptr(recall), N.ptr(ndcg), N.stream_ptr(dev)),
        "hgnn_topk_metrics")
    return topk, recall, ndcg


def recommend(user_emb: torch.Tensor, post_emb: torch.Tensor, K: int = 10,
              batch_scores: int = 1 << 30,
              fused: Optional[bool] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-K posts for every user row: ``(topk_scores, topk_indices)``, each ``[n_users, k]``,
    k = min(K, n_posts) — the scoring of ``recommend_for_user_inductive`` (inference.py:427-429:
    ``torch.topk(user_emb @ known_post_emb.T, min(K, len(scores)))``) for a whole batch of users
    at once.  Scores descend; equal scores list the lower post index first.  ``fused`` (default
    for d in (64, 128), K <= 64): one kernel, no score matrix."""
    dev = N.require_device(user_emb, post_emb)
    if user_emb.dtype != torch.float32 or post_emb.dtype != torch.float32:
        raise TypeError("recommend: fp32 embeddings expected (the reference dtype)")
    n, C = int(user_emb.shape[0]), int(post_emb.shape[0])
    if C == 0:
        raise ValueError("recommend: no posts to rank")
    k = min(K, C)
    d = int(user_emb.shape[1])
    out_s = torch.empty(n, k, dtype=torch.float32, device=dev)
    out_i = torch.empty(n, k, dtype=torch.int32, device=dev)
    if n == 0:
        return out_s, out_i.long()
    lib = N.lib()
    if _fused_ok(d, fused) and k <= 64:
        N.check(lib.hgnn_score_topk(N.ptr(user_emb.contiguous()), None, n,
                                    N.ptr(post_emb.contiguous()), C, d, k, N.ptr(out_s),
                                    N.ptr(out_i), N.stream_ptr(dev)), "hgnn_score_topk")
        return out_s, out_i.long()
    ld = (C + 3) // 4 * 4
    P_c = post_emb.new_zeros(ld, d)
    P_c[:C] = post_emb
    rows = max(1, min(n, batch_scores // ld))
    buf = torch.empty(rows, ld, dtype=torch.float32, device=dev)
    no_rel = torch.zeros(rows + 1, dtype=torch.int32, device=dev)   # empty relevance sets
    scratch = torch.empty(2, rows, dtype=torch.float64, device=dev)
    for r0 in range(0, n, rows):
        r1 = min(n, r0 + rows)
        S = buf[: r1 - r0]
        torch.mm(user_emb[r0:r1], P_c.T, out=S)
        N.check(lib.hgnn_topk_metrics(
            N.ptr(S), r1 - r0, C, ld, N.ptr(no_rel), N.ptr(no_rel), N.ptr(no_rel), K,
            N.ptr(out_i[r0:r1]), N.ptr(scratch[0]), N.ptr(scratch[1]), N.stream_ptr(dev)),
            "hgnn_topk_metrics")
        out_s[r0:r1] = S.gather(1, out_i[r0:r1].long())
    return out_s, out_i.long()
