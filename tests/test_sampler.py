"""Neighbour-sampled mini-batches (sampler.py, csrc/sampler.hip; BASELINE cfg5).

No reference counterpart exists (the reference trains full-batch), so parity is anchored on the
full-graph oracle: with fanouts covering every degree the mini-batch forward must equal the
full-graph forward on the seeds.  With real fanouts, the blocks are checked against a plain-torch
forward/backward over the same sampled edges, and the sampler itself by its defining properties.
"""
import collections

import numpy as np
import pytest
import torch

from oracle import sage_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rand_csr_graph(rng, n_src, n_dst, E):
    src = rng.integers(0, n_src, size=E)
    dst = (n_dst * rng.random(E) ** 2).astype(np.int64)      # skewed in-degrees
    return torch.from_numpy(np.stack([src, dst]).astype(np.int64))


def test_sample_neighbors_properties():
    from truth_recommendation_gnn_amd import graph, sampler
    rng = np.random.default_rng(0)
    ei = _rand_csr_graph(rng, 500, 300, 20000)
    s = sampler.NeighborSampler({"a": 500, "b": 300}, {("a", "r", "b"): ei.to(DEV)},
                                [("a", "r", "b")], [7])
    dst = torch.from_numpy(rng.permutation(300)[:200].astype(np.int32)).to(DEV)
    rp, col = s._sample(("a", "r", "b"), dst, 7, 123)
    rp2, col2 = s._sample(("a", "r", "b"), dst, 7, 123)
    assert torch.equal(rp, rp2) and torch.equal(col, col2)          # deterministic
    _, col3 = s._sample(("a", "r", "b"), dst, 7, 124)
    assert not torch.equal(col, col3)                                # seed-dependent
    nbrs = collections.defaultdict(list)
    for u, v in ei.t().tolist():
        nbrs[v].append(u)
    rp, col = rp.cpu().tolist(), col.cpu().tolist()
    for i, d in enumerate(dst.cpu().tolist()):
        got = col[rp[i]:rp[i + 1]]
        assert len(got) == min(len(nbrs[d]), 7)
        have = collections.Counter(nbrs[d])
        assert not (collections.Counter(got) - have)                 # a sub-multiset
        if len(nbrs[d]) <= 7:
            assert sorted(got) == sorted(nbrs[d])


def test_sample_is_uniform_without_replacement():
    from truth_recommendation_gnn_amd import sampler
    deg, k, trials = 40, 5, 4000
    ei = torch.stack([torch.arange(deg), torch.zeros(deg, dtype=torch.int64)])
    s = sampler.NeighborSampler({"a": deg, "b": 1}, {("a", "r", "b"): ei.to(DEV)},
                                [("a", "r", "b")], [k])
    dst = torch.zeros(1, dtype=torch.int32, device=DEV)
    hits = np.zeros(deg)
    for t in range(trials):
        _, col = s._sample(("a", "r", "b"), dst, k, t)
        c = col.cpu().numpy()
        assert len(set(c.tolist())) == k                              # no repeats
        hits[c] += 1
    expect = trials * k / deg
    assert np.abs(hits - expect).max() < 5 * np.sqrt(expect)          # ~uniform


def test_relabel_prefix_then_new_ids_in_first_appearance_order():
    from truth_recommendation_gnn_amd import sampler
    rng = np.random.default_rng(1)
    n = 1000
    prefix = rng.permutation(n)[:50].astype(np.int32)
    items = rng.integers(0, n, size=3000).astype(np.int32)
    items[:40] = prefix[:40]
    ei = torch.zeros(2, 1, dtype=torch.int64, device=DEV)
    s = sampler.NeighborSampler({"a": n}, {("a", "r", "a"): ei}, [("a", "r", "a")], [3])
    nodes, local, count = s._relabel("a", torch.from_numpy(prefix).to(DEV),
                                     torch.from_numpy(items).to(DEV))
    nodes, local = nodes[:int(count[0])].cpu().numpy(), local.cpu().numpy()
    assert np.array_equal(nodes[:50], prefix)
    pre = set(prefix.tolist())
    new = list(dict.fromkeys(i for i in items.tolist() if i not in pre))
    assert nodes[50:].tolist() == new
    assert np.array_equal(nodes[local], items)


def _cfg5_tiny():
    from truth_recommendation_gnn_amd import synth
    cfg = synth.scaled("cfg5", 0.00004)           # 360 users, 40 posts, 8k engages, 4 relations
    cfg = synth.dataclasses.replace(cfg, dim=16, hidden=16)
    g = synth.make_graph(cfg)
    rels = [(synth.REV_ENGAGES, 1.0), (synth.SOCIAL, 0.75), (synth.ENGAGES, 1.0),
            (synth.POST_POST, 0.5)]
    return cfg, g, rels


def _model(cfg, rels):
    from truth_recommendation_gnn_amd import HeteroSAGE
    names = []
    for l in range(2):
        for et, _ in rels:
            p = f"layers.{l}.{'__'.join(et)}"
            names += [(f"{p}.lin_l.weight", (16, 16)), (f"{p}.lin_l.bias", (16,)),
                      (f"{p}.lin_r.weight", (16, 16))]
    params = sage_ref.init_params(names)
    m = HeteroSAGE(16, rels, num_layers=2).to(DEV)
    m.load_state_dict(params)
    return m, params


def test_full_fanout_minibatch_equals_full_graph_forward():
    from truth_recommendation_gnn_amd import sampler
    cfg, g, rels = _cfg5_tiny()
    model, params = _model(cfg, rels)
    num = {"user": cfg.num_users, "post": cfg.num_posts}
    ei = {et: e.to(DEV) for et, e in g.edge_index_dict.items()}
    s = sampler.NeighborSampler(num, ei, [et for et, _ in rels], [-1, -1])
    seeds = {"user": torch.arange(0, cfg.num_users, 7), "post": torch.arange(0, cfg.num_posts, 3)}
    mb = s.sample(seeds, seed=5)
    x = {t: v.to(DEV) for t, v in g.x_dict.items()}
    got = sampler.forward_blocks(model, mb, x)
    ref = sage_ref.hetero_sage(params, g.x_dict, g.edge_index_dict, rels, 2)
    for t, ids in seeds.items():
        r = ref[t][ids]
        torch.testing.assert_close(got[t].cpu(), r, rtol=1e-4, atol=1e-5 * float(r.abs().max()))


def _torch_blocks(params, rels, mb, x):
    """Plain-torch forward over the same sampled blocks (CPU): the check for fanout < degree."""
    h = {t: x[t][ids.long().cpu()] for t, ids in mb.nodes[0].items()}
    for l, blk in enumerate(mb.blocks):
        out = {}
        for dst, n_dst in blk.n_dst.items():
            acc = None
            for et, w in rels:
                if et[2] != dst or et not in blk.csr:
                    continue
                ei = blk.csr[et].edge_index.cpu()
                wl, bl, wr = sage_ref._conv_params(params, f"layers.{l}.{'__'.join(et)}")
                m = sage_ref.sage_conv(h[et[0]], h[dst][:n_dst], ei, wl, bl, wr)
                acc = w * m if acc is None else acc + w * m
            out[dst] = torch.relu(acc) if acc is not None else h[dst][:n_dst]
        h = out
    return h


def test_sampled_minibatch_forward_backward_match_torch_on_blocks():
    from truth_recommendation_gnn_amd import sampler
    cfg, g, rels = _cfg5_tiny()
    model, params = _model(cfg, rels)
    num = {"user": cfg.num_users, "post": cfg.num_posts}
    ei = {et: e.to(DEV) for et, e in g.edge_index_dict.items()}
    s = sampler.NeighborSampler(num, ei, [et for et, _ in rels], [5, 3])
    seeds = {"user": torch.arange(3, cfg.num_users, 11), "post": torch.arange(0, cfg.num_posts, 4)}
    mb = s.sample(seeds, seed=9)
    assert all(b.csr[et].num_edges <= 5 * b.n_dst[et[2]] for b in mb.blocks[1:] for et in b.csr)
    x = {t: v.to(DEV) for t, v in g.x_dict.items()}
    got = sampler.forward_blocks(model, mb, x)
    ref_params = {k: v.clone().requires_grad_() for k, v in params.items()}
    ref = _torch_blocks(ref_params, rels, mb, g.x_dict)
    gen = torch.Generator().manual_seed(0)
    wts = {t: torch.randn(ref[t].shape, generator=gen) for t in ref}
    loss = sum((got[t] * wts[t].to(DEV)).sum() for t in got)
    loss.backward()
    ref_loss = sum((ref[t] * wts[t]).sum() for t in ref)
    ref_loss.backward()
    for t in ref:
        torch.testing.assert_close(got[t].detach().cpu(), ref[t].detach(), rtol=1e-4,
                                   atol=1e-5 * float(ref[t].detach().abs().max()))
    for name, p in model.named_parameters():
        r = ref_params[name].grad
        torch.testing.assert_close(p.grad.cpu(), r, rtol=1e-4, atol=1e-5 * float(r.abs().max()))


def test_sampled_blocks_with_hot_sources_backward_matches_torch():
    """A source drawn by more sampled edges than the default split chunk (64): the blocks carry
    no skew plan, so such a CSC row must be summed whole (a hot post under many seed users: at
    cfg5 700+ of one block's rev_engages edges).  Regression: it was skipped as 'heavy'."""
    from truth_recommendation_gnn_amd import HeteroSAGE, sampler, synth
    rng = np.random.default_rng(4)
    n_u, n_p = 600, 12
    users = np.concatenate([np.arange(n_u), rng.integers(0, n_u, 900)])
    posts = np.concatenate([np.zeros(n_u, dtype=np.int64), rng.integers(1, n_p, 900)])
    eng = torch.from_numpy(np.stack([users, posts]).astype(np.int64))
    ei = {synth.ENGAGES: eng.to(DEV), synth.REV_ENGAGES: eng.flip(0).contiguous().to(DEV)}
    rels = [(synth.REV_ENGAGES, 1.0), (synth.ENGAGES, 1.0)]
    names = []
    for l in range(2):
        for et, _ in rels:
            p = f"layers.{l}.{'__'.join(et)}"
            names += [(f"{p}.lin_l.weight", (16, 16)), (f"{p}.lin_l.bias", (16,)),
                      (f"{p}.lin_r.weight", (16, 16))]
    params = sage_ref.init_params(names)
    model = HeteroSAGE(16, rels, num_layers=2).to(DEV)
    model.load_state_dict(params)
    s = sampler.NeighborSampler({"user": n_u, "post": n_p}, ei, [et for et, _ in rels], [8, 8])
    seeds = {"user": torch.arange(0, n_u, 2), "post": torch.arange(0, n_p)}
    mb = s.sample(seeds, seed=2)
    hot = int(torch.bincount(mb.blocks[-1].csr[synth.REV_ENGAGES].edge_index[0]).max())
    assert hot > 64
    gen = torch.Generator().manual_seed(3)
    x = {"user": torch.randn(n_u, 16, generator=gen), "post": torch.randn(n_p, 16, generator=gen)}
    got = sampler.forward_blocks(model, mb, {t: v.to(DEV) for t, v in x.items()})
    ref_params = {k: v.clone().requires_grad_() for k, v in params.items()}
    ref = _torch_blocks(ref_params, rels, mb, x)
    wts = {t: torch.randn(ref[t].shape, generator=gen) for t in ref}
    sum((got[t] * wts[t].to(DEV)).sum() for t in got).backward()
    sum((ref[t] * wts[t]).sum() for t in ref).backward()
    for name, p in model.named_parameters():
        r = ref_params[name].grad
        torch.testing.assert_close(p.grad.cpu(), r, rtol=1e-4,
                                   atol=1e-5 * float(r.abs().max()), msg=name)


def test_relabel_edge_cases_and_seed_checks():
    from truth_recommendation_gnn_amd import sampler
    ei = torch.tensor([[0, 1, 2], [1, 2, 0]], device=DEV)
    s = sampler.NeighborSampler({"a": 3}, {("a", "r", "a"): ei}, [("a", "r", "a")], [2])
    pre = torch.tensor([2, 0], dtype=torch.int32, device=DEV)
    none = torch.empty(0, dtype=torch.int32, device=DEV)
    nodes, local, count = s._relabel("a", pre, none)                  # no items
    assert int(count[0]) == 2 and nodes[:2].tolist() == [2, 0] and local.numel() == 0
    nodes, local, count = s._relabel("a", none, torch.tensor([5, 5, 3, 9, 3], dtype=torch.int32,
                                                               device=DEV))   # no prefix
    assert int(count[0]) == 3 and nodes[:3].tolist() == [5, 3, 9] and local.tolist() == [0, 0, 1, 2, 1]
    with pytest.raises(ValueError, match="distinct"):
        s.sample({"a": torch.tensor([0, 0])})
    with pytest.raises(ValueError, match="out of range"):
        s.sample({"a": torch.tensor([3])})
    mb = s.sample({"a": torch.tensor([1])}, seed=1)
    assert mb.nodes[-1]["a"].tolist() == [1]
    with pytest.raises(ValueError, match="out of range"):   # far outside: degree 0, no read
        s.sample({"a": torch.tensor([1, 10**6])})
    with pytest.raises(ValueError, match="out of range"):
        s.sample({"a": torch.tensor([-1])})
    with pytest.raises(ValueError, match="distinct"):      # a repeat among many seeds
        s.sample({"a": torch.tensor([2, 0, 1, 0])})
    # the flags are per call: a clean batch after a bad one samples normally
    mb = s.sample({"a": torch.tensor([2, 0])}, seed=3)
    assert mb.nodes[-1]["a"].tolist() == [2, 0]


@pytest.mark.parametrize("n_src,n_dst,E", [(1, 1, 1), (37, 11, 500), (5000, 300, 60000),
                                           (300, 5000, 7000)])
def test_csr_transpose_equals_coo_grouping(n_src, n_dst, E):
    """hgnn_csr_transpose (a from_csr relation's CSC, sampled blocks) against the CSC that
    group_edges builds from the COO: same rowptr, rows and positions (stable), and 1/deg(row)
    per entry equal to inv_deg[row]."""
    from truth_recommendation_gnn_amd import graph
    rng = np.random.default_rng(n_src + E)
    ei = _rand_csr_graph(rng, n_src, n_dst, E).to(DEV)
    full = graph.RelationCSR(ei, n_src, n_dst)
    blk = graph.RelationCSR.from_csr(full.fwd.rowptr, full.fwd.col, n_src, n_dst,
                                     may_have_heavy_rows=False)
    want = graph.group_edges(full.fwd.col.long(), blk._dst_of_positions(torch.int64), n_src,
                             n_dst)
    got = blk.bwd
    assert torch.equal(got.rowptr, want.rowptr)
    assert torch.equal(got.col, want.col)
    assert torch.equal(got.perm, want.perm)
    assert torch.equal(blk.bwd_weights, full.inv_deg[got.col.long()])


@pytest.mark.parametrize("fanout", [3, 10, -1])
def test_hop_batch_equals_per_relation_sampling(fanout):
    """hgnn_sample_hop_count/_fill (every relation of a hop in one launch per phase) give, per
    relation, exactly the rowptr and sample of hgnn_sample_neighbors on its own — including a
    relation with no destinations and ids outside the table (counted as degree 0)."""
    from truth_recommendation_gnn_amd import sampler
    rng = np.random.default_rng(7)
    ei = {("a", "r1", "b"): _rand_csr_graph(rng, 400, 300, 9000),
          ("b", "r2", "b"): _rand_csr_graph(rng, 300, 300, 4000),
          ("a", "r3", "a"): _rand_csr_graph(rng, 400, 400, 100),
          ("b", "r4", "a"): _rand_csr_graph(rng, 300, 400, 7000)}
    ets = list(ei)
    s = sampler.NeighborSampler({"a": 400, "b": 300}, {k: v.to(DEV) for k, v in ei.items()},
                                ets, [fanout])
    cur = {"b": torch.from_numpy(rng.permutation(300)[:120].astype(np.int32)).to(DEV),
           "a": torch.empty(0, dtype=torch.int32, device=DEV)}
    rowptr, cols, totals = s._hop(ets, cur, fanout, 99)
    o = 0
    for et in ets:
        rp, col = s._sample(et, cur[et[2]], fanout, 99)
        assert torch.equal(rowptr[et], rp), et
        assert totals[et] == int(rp[-1])
        assert torch.equal(cols[o:o + totals[et]], col), et
        o += totals[et]
    bad = {"b": torch.tensor([5, 300, -2, 7], dtype=torch.int32, device=DEV)}
    rowptr, cols, totals = s._hop([("a", "r1", "b")], bad, fanout, 1)
    deg = rowptr[("a", "r1", "b")].diff().tolist()
    assert deg[1] == 0 and deg[2] == 0


def test_relabel_multi_equals_per_type_relabel():
    """hgnn_relabel_multi (every type of a hop in one call, table keyed by id x types + type)
    gives each type the node set and local ids of its own hgnn_relabel call — the same id in two
    types stays two nodes."""
    from truth_recommendation_gnn_amd import sampler
    rng = np.random.default_rng(9)
    num = {"a": 700, "b": 300, "c": 50}
    ei = torch.zeros(2, 1, dtype=torch.int64, device=DEV)
    s = sampler.NeighborSampler(num, {("a", "r", "a"): ei}, [("a", "r", "a")], [3])
    types = ["a", "b", "c"]
    cur = {"a": torch.from_numpy(rng.permutation(700)[:40].astype(np.int32)).to(DEV),
           "b": torch.from_numpy(rng.permutation(300)[:25].astype(np.int32)).to(DEV)}
    items = {"a": rng.integers(0, 300, 2000), "b": rng.integers(0, 300, 900),
             "c": rng.integers(0, 50, 70)}                  # "a" ids overlap "b" ids
    items["a"][:30] = cur["a"][:30].cpu().numpy()
    allit = torch.from_numpy(np.concatenate([items[t] for t in types]).astype(np.int32)).to(DEV)
    n_items = [len(items[t]) for t in types]
    nodes, local, counts = s._relabel_hop(types, cur, allit, n_items)
    counts = counts.tolist()
    o = 0
    for i, t in enumerate(types):
        pre = cur.get(t, torch.empty(0, dtype=torch.int32, device=DEV))
        it = allit[o:o + n_items[i]]
        n1, l1, c1 = s._relabel(t, pre, it)
        assert counts[2 * i] == int(c1[0]) and counts[2 * i + 1] == 0
        assert torch.equal(nodes[t][:counts[2 * i]], n1[:int(c1[0])]), t
        assert torch.equal(local[o:o + n_items[i]], l1), t
        o += n_items[i]


def test_block_csc_group_equals_per_relation_transpose():
    """The CSCs of a sampled block's relations built together (hgnn_csr_transpose_multi, one
    sort) equal the per-relation hgnn_csr_transpose: rowptr, rows, positions and K2 weights —
    including a relation with no edges."""
    from truth_recommendation_gnn_amd import graph
    rng = np.random.default_rng(11)
    specs = [(300, 120, 4000), (50, 120, 0), (700, 80, 9000), (120, 300, 2500)]
    rels_a, rels_b = [], []
    for n_src, n_dst, E in specs:
        ei = _rand_csr_graph(rng, n_src, n_dst, E).to(DEV) if E else \
            torch.zeros(2, 0, dtype=torch.int64, device=DEV)
        full = graph.RelationCSR(ei, n_src, n_dst)
        for out in (rels_a, rels_b):
            out.append(graph.RelationCSR.from_csr(full.fwd.rowptr, full.fwd.col, n_src, n_dst,
                                                  may_have_heavy_rows=False))
    graph.build_csc_group(rels_a)
    for a, b in zip(rels_a, rels_b):
        ga, gb = a.bwd, b.bwd                     # b: the one-relation transpose
        assert torch.equal(ga.rowptr, gb.rowptr)
        assert torch.equal(ga.col, gb.col) and torch.equal(ga.perm, gb.perm)
        assert torch.equal(a.bwd_weights, b.bwd_weights)


@pytest.mark.parametrize("case", ["empty", "empty_both", "zero_degree_users", "zero_degree_posts",
                                  "posts_only", "mixed"])
def test_edge_case_seed_sets_match_full_graph(case):
    """Empty seed sets, seeds with no in-neighbours (their SAGE output is lin_r(x) + bias), and a
    seed dict naming one of two types: with fanouts covering every degree the mini-batch equals
    the full-graph oracle on the seeds, and its backward runs (zero-row blocks included)."""
    from truth_recommendation_gnn_amd import HeteroSAGE, sampler
    e = lambda *v: torch.tensor(v, dtype=torch.int64)               # noqa: E731
    ei = {("user", "engages", "post"): torch.stack([e(0, 1, 2, 3), e(0, 0, 1, 1)]),  # posts 2, 3: deg 0
          ("post", "rev", "user"): torch.stack([e(0, 1), e(0, 2)])}                 # users 1, 3, 4: deg 0
    rels = [(et, w) for et, w in zip(ei, (1.0, 0.75))]
    seeds = {"empty": {"user": e()}, "empty_both": {"user": e(), "post": e()},
             "zero_degree_users": {"user": e(1, 3, 4)}, "zero_degree_posts": {"post": e(2, 3)},
             "posts_only": {"post": e(0, 1)}, "mixed": {"user": e(0), "post": e(3)}}[case]
    names = [(f"layers.{l}.{'__'.join(et)}.{n}", s) for l in range(2) for et in ei
             for n, s in (("lin_l.weight", (8, 8)), ("lin_l.bias", (8,)), ("lin_r.weight", (8, 8)))]
    params = sage_ref.init_params(names)
    model = HeteroSAGE(8, rels, num_layers=2).to(DEV)
    model.load_state_dict(params)
    x = {"user": torch.randn(5, 8, generator=torch.Generator().manual_seed(0)),
         "post": torch.randn(4, 8, generator=torch.Generator().manual_seed(1))}
    s = sampler.NeighborSampler({"user": 5, "post": 4}, {et: v.to(DEV) for et, v in ei.items()},
                                list(ei), [-1, 2])
    mb = s.sample(seeds, seed=1)
    got = sampler.forward_blocks(model, mb, {t: v.to(DEV) for t, v in x.items()})
    ref = sage_ref.hetero_sage(params, x, ei, rels, 2)
    assert set(got) == set(seeds)
    for t, ids in seeds.items():
        assert got[t].shape == (ids.numel(), 8)
        torch.testing.assert_close(got[t].cpu(), ref[t][ids], rtol=1e-5, atol=1e-6)
    loss = sum(v.sum() for v in got.values())
    if loss.requires_grad:
        loss.backward()
        assert all(torch.isfinite(p.grad).all() for p in model.parameters() if p.grad is not None)
