"""BASELINE cfg5 at full size (9M users, 1M posts, 200M engages + reverse, 90M follows, 10M
post -> post edges, d = h = 128; fanout [15, 10], 1024 + 1024 seeds): one neighbour-sampled
mini-batch, the configuration bench.py's ``--config cfg5`` line times.

No reference counterpart exists (the reference trains full-batch, train_gnn.py:254), so the batch
is checked by what defines it:
* the sampler: every sampled edge is an edge of the graph (as a multiset per destination: no
  position drawn twice), each destination keeps min(degree, fanout) of its in-edges, and block
  l's destinations are the first nodes of its sources (PyG NeighborLoader's relabel order);
* the HIP forward / backward over the blocks (K1/K2/K3 on the sampled CSRs) against plain torch
  on the same blocks (tests/test_sampler.py's ``_torch_blocks``): outputs and every parameter
  gradient at rtol 1e-4.
"""
import numpy as np
import pytest
import torch

from oracle import sage_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
FANOUTS = [15, 10]


@pytest.fixture(scope="module")
def cfg5():
    from truth_recommendation_gnn_amd import sampler, synth
    cfg = synth.CONFIGS["cfg5"]
    g = synth.make_graph(cfg, device=DEV, device_gen=True)
    rels = [(synth.REV_ENGAGES, 1.0), (synth.SOCIAL, 0.75), (synth.ENGAGES, 1.0),
            (synth.POST_POST, 0.5)]
    num = {"user": cfg.num_users, "post": cfg.num_posts}
    s = sampler.NeighborSampler(num, g.edge_index_dict, [et for et, _ in rels], FANOUTS)
    gen = torch.Generator(device=DEV).manual_seed(17)
    seeds = {"user": torch.randperm(cfg.num_users, device=DEV, generator=gen)[:1024],
             "post": torch.randperm(cfg.num_posts, device=DEV, generator=gen)[:1024]}
    mb = s.sample(seeds, seed=3)
    yield cfg, g, rels, num, seeds, mb
    del g, s, mb
    torch.cuda.empty_cache()


class _Rows:
    """Row indexing into a device table that hands the rows back on the host."""

    def __init__(self, t):
        self.t = t

    def __getitem__(self, idx):
        return self.t[idx.to(self.t.device)].cpu()


def _multiset_subset(sampled_keys, graph_keys_sorted):
    """Every sampled key occurs in the graph at least as often as in the sample."""
    u, c = torch.unique(sampled_keys, return_counts=True)
    lo = torch.searchsorted(graph_keys_sorted, u, right=False)
    hi = torch.searchsorted(graph_keys_sorted, u, right=True)
    return bool(((hi - lo) >= c).all())


def test_cfg5_sampled_blocks_are_graph_edges_with_fanout(cfg5):
    cfg, g, rels, num, seeds, mb = cfg5
    for t, ids in seeds.items():                       # the last frontier is the seeds, in order
        assert torch.equal(mb.nodes[-1][t].long(), ids.long())
    n_sampled = 0
    for l, blk in enumerate(mb.blocks):
        fan = FANOUTS[len(mb.blocks) - 1 - l]          # blocks[-1] is the seeds' hop
        for t, n in blk.n_dst.items():                 # destinations = a prefix of the sources
            assert torch.equal(mb.nodes[l][t][:n], mb.nodes[l + 1][t])
        for et, csr in blk.csr.items():
            src_t, _, dst_t = et
            ei = csr.edge_index                        # local ids
            src = mb.nodes[l][src_t].long()[ei[0].long()]
            dst = mb.nodes[l + 1][dst_t].long()[ei[1].long()]
            n_src_glob = num[src_t]
            full = g.edge_index_dict[et]
            gkeys = torch.sort(full[1] * n_src_glob + full[0])[0]
            assert _multiset_subset(dst * n_src_glob + src, gkeys), et
            # per destination: min(in-degree, fanout) sampled in-edges
            deg = torch.bincount(full[1], minlength=num[dst_t])
            want = torch.clamp(deg[mb.nodes[l + 1][dst_t].long()], max=fan)
            got = torch.bincount(ei[1].long(), minlength=blk.n_dst[dst_t])
            assert torch.equal(got, want), et
            n_sampled += int(ei.shape[1])
    assert n_sampled > 100_000                          # a real batch, not a degenerate one


def test_cfg5_minibatch_forward_backward_match_torch_on_blocks(cfg5):
    import test_sampler
    from truth_recommendation_gnn_amd import HeteroSAGE, sampler
    cfg, g, rels, num, seeds, mb = cfg5
    names = []
    for l in range(cfg.layers):
        for et, _ in rels:
            p = f"layers.{l}.{'__'.join(et)}"
            names += [(f"{p}.lin_l.weight", (cfg.hidden, cfg.dim)),
                      (f"{p}.lin_l.bias", (cfg.hidden,)),
                      (f"{p}.lin_r.weight", (cfg.hidden, cfg.dim))]
    params = sage_ref.init_params(names)
    model = HeteroSAGE(cfg.hidden, rels, num_layers=cfg.layers, in_channels=cfg.dim).to(DEV)
    model.load_state_dict(params)
    got = sampler.forward_blocks(model, mb, g.x_dict)
    # the torch reference reads only the batch's input rows (the 4.6 GB table stays on the GPU)
    x_in = {t: _Rows(g.x_dict[t]) for t in mb.nodes[0]}
    ref_params = {k: v.clone().requires_grad_() for k, v in params.items()}
    ref = test_sampler._torch_blocks(ref_params, rels, mb, x_in)
    gen = torch.Generator().manual_seed(1)
    wts = {t: torch.randn(ref[t].shape, generator=gen) for t in ref}
    (sum((got[t] * wts[t].to(DEV)).sum() for t in got)).backward()
    (sum((ref[t] * wts[t]).sum() for t in ref)).backward()
    for t in ref:
        r = ref[t].detach()
        torch.testing.assert_close(got[t].detach().cpu(), r, rtol=1e-4,
                                   atol=1e-5 * float(r.abs().max()))
    for name, p in model.named_parameters():
        r = ref_params[name].grad
        torch.testing.assert_close(p.grad.cpu(), r, rtol=1e-4,
                                   atol=1e-5 * max(float(r.abs().max()), 1e-12), msg=name)
