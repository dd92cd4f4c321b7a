"""Batched Recall@K / NDCG@K (train_gnn.py:289-367): the HIP kernel (csrc/eval.hip) against the
reference loop restated in oracle/eval_ref.py, whose NDCG is sklearn's own ndcg_score."""
import math

import numpy as np
import pytest
import torch
from sklearn.metrics import ndcg_score

from oracle import eval_ref

DEV = torch.device("cuda")


def tie_averaged_ndcg(scores, rel, k):
    """The group formula the kernel implements: entries with equal score form a group that
    shares its mean gain over the group's rank positions (cut at k)."""
    vals = sorted(set(scores.tolist()), reverse=True)
    disc = [1.0 / math.log2(i + 2) for i in range(len(scores))]
    dcg, start = 0.0, 0
    for v in vals:
        members = [i for i, s in enumerate(scores) if s == v]
        n, r = len(members), sum(rel[i] for i in members)
        dcg += r / n * sum(disc[start:min(start + n, k)])
        start += n
        if start >= k:
            break
    m = int(sum(rel))
    idcg = sum(disc[:min(k, m)])
    return dcg / idcg if idcg > 0 else 0.0


@pytest.mark.parametrize("seed", range(8))
def test_tie_averaged_formula_is_sklearns(seed):
    rng = np.random.default_rng(seed)
    C = int(rng.integers(2, 40))
    scores = rng.integers(-3, 4, size=C).astype(np.float32)    # heavy ties, incl. at the cut
    rel = (rng.random(C) < 0.3).astype(np.float64)
    if rel.sum() == 0:
        rel[int(rng.integers(0, C))] = 1.0
    for k in (1, 3, 10, C + 5):
        ref = ndcg_score(rel.reshape(1, -1), scores.reshape(1, -1), k=k)
        assert abs(tie_averaged_ndcg(scores, rel, k) - ref) < 1e-12


def test_oracle_tie_break_only_moves_boundary_ties():
    g = torch.Generator().manual_seed(1)
    U = torch.randn(30, 8, generator=g)
    P = torch.randn(40, 8, generator=g)
    te = torch.stack([torch.randint(0, 30, (200,), generator=g),
                      torch.randint(30, 70, (200,), generator=g)])
    a = eval_ref.evaluate(te, U, P, 30, K=10)
    b = eval_ref.evaluate(te, U, P, 30, K=10, tie_break="index")
    assert a == b   # continuous scores: no ties, both orders agree


# ----------------------------------------------------------------------------- GPU
def _int_case(seed, n_users, n_posts, E, d, lo=-2, hi=3, extra_users=0):
    """Integer embeddings: fp32 dot products are exact, so CPU and GPU scores are identical
    and full of ties."""
    rng = np.random.default_rng(seed)
    U = torch.from_numpy(rng.integers(lo, hi, size=(n_users, d)).astype(np.float32))
    P = torch.from_numpy(rng.integers(lo, hi, size=(n_posts, d)).astype(np.float32))
    u = rng.integers(0, n_users + extra_users, size=E)
    p = n_users + rng.integers(0, n_posts, size=E)
    u[: E // 10] = u[E // 10: 2 * (E // 10)]     # duplicate test edges
    p[: E // 10] = p[E // 10: 2 * (E // 10)]
    return U, P, torch.from_numpy(np.stack([u, p]).astype(np.int64))


@pytest.mark.gpu
@pytest.mark.parametrize("d,fused", [(8, False), (64, True), (64, False), (128, True)])
@pytest.mark.parametrize("n_users,n_posts,E,K", [(300, 257, 3000, 10), (64, 7, 200, 10),
                                                 (500, 1000, 2500, 1), (200, 90, 800, 33),
                                                 (150, 700, 1500, 63)])
def test_evaluate_matches_reference_loop_exact_scores(n_users, n_posts, E, K, d, fused):
    """Integer embeddings: exact scores, full of ties — on the fused path most rows are redone
    on the materialised one (tie across the cut), the rest finish from the fused lists."""
    from truth_recommendation_gnn_amd import evaluate
    U, P, te = _int_case(n_users + K, n_users, n_posts, E, d, extra_users=5)
    users, rec, nd = eval_ref.evaluate(te, U, P, n_users, K=K, tie_break="index", per_user=True)
    r, n = evaluate(te.to(DEV), U.to(DEV), P.to(DEV), K=K, fused=fused)
    assert abs(r - float(np.mean(rec))) < 1e-12
    assert abs(n - float(np.mean(nd))) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("d", [64, 128])
def test_fused_evaluate_without_ties_matches_reference(d):
    """Distinct scores (integer embeddings from a wide range): no row needs the tie pass, every
    metric comes from the fused lists."""
    from truth_recommendation_gnn_amd import evaluate
    U, P, te = _int_case(d, 400, 3000, 6000, d, lo=-60, hi=61)
    users, rec, nd = eval_ref.evaluate(te, U, P, 400, K=10, tie_break="index", per_user=True)
    r, n = evaluate(te.to(DEV), U.to(DEV), P.to(DEV), K=10, fused=True)
    assert abs(r - float(np.mean(rec))) < 1e-12
    assert abs(n - float(np.mean(nd))) < 1e-12


@pytest.mark.gpu
def test_topk_metrics_rows_match_python_ranking():
    from truth_recommendation_gnn_amd import metrics
    rng = np.random.default_rng(7)
    rows, C, K = 37, 203, 12
    S = rng.integers(-4, 5, size=(rows, C)).astype(np.float32)
    rel_sets = [sorted(set(rng.integers(0, C, size=int(rng.integers(1, 9))).tolist()))
                for _ in range(rows)]
    counts = [len(s) + int(rng.integers(0, 3)) for s in rel_sets]
    rowptr = np.concatenate([[0], np.cumsum([len(s) for s in rel_sets])]).astype(np.int32)
    tc = np.concatenate(rel_sets).astype(np.int32)
    topk, rec, nd = metrics.topk_metrics(torch.from_numpy(S).to(DEV),
                                         torch.from_numpy(rowptr).to(DEV),
                                         torch.from_numpy(tc).to(DEV),
                                         torch.tensor(counts, dtype=torch.int32, device=DEV), K)
    for i in range(rows):
        order = sorted(range(C), key=lambda j: (-S[i, j], j))[:K]
        assert topk[i].tolist() == order
        rel = np.zeros(C)
        rel[rel_sets[i]] = 1.0
        hits = len(set(order) & set(rel_sets[i]))
        assert float(rec[i]) == hits / counts[i]
        assert abs(float(nd[i]) - ndcg_score(rel.reshape(1, -1), S[i:i + 1], k=K)) < 1e-12


@pytest.mark.gpu
def test_evaluate_continuous_embeddings():
    from truth_recommendation_gnn_amd import evaluate
    g = torch.Generator().manual_seed(3)
    U = torch.nn.functional.normalize(torch.randn(400, 64, generator=g), dim=1)
    P = torch.nn.functional.normalize(torch.randn(500, 64, generator=g), dim=1)
    te = torch.stack([torch.randint(0, 400, (4000,), generator=g),
                      400 + torch.randint(0, 500, (4000,), generator=g)])
    ref = eval_ref.evaluate(te, U, P, 400, K=10)
    got = evaluate(te.to(DEV), U.to(DEV), P.to(DEV), K=10, batch_scores=64 * 500)   # 8 batches
    # fp32 GEMM vs CPU mm may reorder near-equal scores: allow a couple of boundary swaps
    assert abs(got[0] - ref[0]) < 2e-3
    assert abs(got[1] - ref[1]) < 2e-3


@pytest.mark.gpu
def test_evaluate_edge_cases():
    from truth_recommendation_gnn_amd import evaluate
    U = torch.ones(3, 4, device=DEV)
    P = torch.ones(2, 4, device=DEV)
    empty = torch.empty(2, 0, dtype=torch.int64, device=DEV)
    r, n = evaluate(empty, U, P)
    assert math.isnan(r) and math.isnan(n)
    only_bad_users = torch.tensor([[7, 9], [3, 4]], device=DEV)     # users >= num_users skipped
    r, n = evaluate(only_bad_users, U, P)
    assert math.isnan(r)
    with pytest.raises(ValueError):
        evaluate(torch.tensor([[0], [1]], device=DEV), U, P)        # post id < num_users


@pytest.mark.gpu
@pytest.mark.parametrize("d", [16, 64, 128])
@pytest.mark.parametrize("n,C,K", [(50, 1000, 10), (3, 7, 10), (300, 4097, 25), (129, 65, 63)])
def test_recommend_matches_topk(n, C, K, d):
    """inference.py:427-429: torch.topk over user_emb @ known_post_emb.T, batched over users
    (d 64/128: the fused kernel; 16: the materialised path)."""
    from truth_recommendation_gnn_amd import recommend
    rng = np.random.default_rng(C)
    U = torch.from_numpy(rng.integers(-3, 4, size=(n, d)).astype(np.float32))
    P = torch.from_numpy(rng.integers(-3, 4, size=(C, d)).astype(np.float32))
    S = U @ P.T                                   # exact (integers): CPU == GPU scores
    s, i = recommend(U.to(DEV), P.to(DEV), K, batch_scores=64 * C)
    k = min(K, C)
    assert s.shape == (n, k) and i.shape == (n, k)
    for r in range(n):
        order = sorted(range(C), key=lambda j: (-float(S[r, j]), j))[:k]
        assert i[r].tolist() == order
        assert torch.equal(s[r].cpu(), S[r, order])
    # ties aside, the same multiset of scores as torch.topk (what the reference returns)
    ts, _ = torch.topk(S, k, dim=1)
    assert torch.equal(s.cpu(), ts)
