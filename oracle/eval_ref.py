"""CPU ORACLE — test infrastructure only, never the product path.

Restatement of the reference's evaluation loop ``evaluate(test_edges, user_emb, post_emb, K=10)``
(``train_gnn.py:289-367``), user by user exactly as written there:

* test edges grouped per user in first-appearance order (``train_gnn.py:313-318``), global post
  ids made local with ``p - num_users`` (the reference's module-level ``num_users``);
* candidates = the sorted set of every test post (``train_gnn.py:320-322``);
* users ``>= num_users`` skipped (``train_gnn.py:328-329``);
* scores = ``user_emb[u] @ post_emb[candidates].T`` in fp32 (``train_gnn.py:335-338``), top
  ``min(K, C)`` (``train_gnn.py:341-342``);
* Recall = |set(top-K posts) & set(true_posts)| / len(true_posts) — len counts duplicate test
  edges (``train_gnn.py:345-347``);
* NDCG = ``sklearn.metrics.ndcg_score(relevance, scores, k=K)`` on binary relevance over the
  candidates (``train_gnn.py:350-364``) — sklearn is installed here, so the reference's own
  metric code computes it (default ``ignore_ties=False``: tie-averaged DCG);
* the means over users (``train_gnn.py:367``).

The only liberty: ``torch.topk``'s choice among equal scores at the K boundary is unspecified, so
``tie_break="index"`` (optional) takes the lower candidate index, as the HIP kernel does; the
default uses ``torch.topk`` itself.  NDCG does not depend on that choice (sklearn ranks by score).

PARITY STATUS: the loop is the reference's; sklearn's ndcg_score is the reference's own metric.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch
from sklearn.metrics import ndcg_score


def evaluate(test_edges: torch.Tensor, user_emb: torch.Tensor, post_emb: torch.Tensor,
             num_users: int, K: int = 10, tie_break: str = "torch", per_user: bool = False):
    te = test_edges.cpu()
    U, P = user_emb.detach().cpu().float(), post_emb.detach().cpu().float()
    user_test_posts: "OrderedDict[int, list]" = OrderedDict()
    cand_set = set()
    for i in range(te.shape[1]):
        u = int(te[0, i])
        p_local = int(te[1, i]) - num_users
        user_test_posts.setdefault(u, []).append(p_local)
        cand_set.add(p_local)
    cand = torch.tensor(sorted(cand_set), dtype=torch.int64)
    recall_list, ndcg_list, users = [], [], []
    for u, true_posts in user_test_posts.items():
        if u >= num_users or not true_posts:
            continue
        scores = torch.mm(U[u].unsqueeze(0), P[cand].T).squeeze(0)
        k = min(K, len(scores))
        if tie_break == "index":
            order = sorted(range(len(scores)), key=lambda j: (-float(scores[j]), j))
            topk_idx = torch.tensor(order[:k])
        else:
            topk_idx = torch.topk(scores, k)[1]
        topk_posts = cand[topk_idx].tolist()
        hits = len(set(topk_posts) & set(true_posts))
        recall_list.append(hits / len(true_posts))
        relevance = torch.zeros(len(cand))
        for p in true_posts:
            idx = (cand == p).nonzero(as_tuple=True)[0]
            if len(idx) > 0:
                relevance[idx] = 1.0
        if relevance.sum() > 0:
            ndcg_list.append(ndcg_score(relevance.numpy().reshape(1, -1),
                                        scores.numpy().reshape(1, -1), k=K))
        users.append(u)
    if per_user:
        return users, recall_list, ndcg_list
    return float(np.mean(recall_list)), float(np.mean(ndcg_list))
