"""Test cases shared by the CPU (gloo) and GPU distributed tests: small seeded graphs, the
model, its seeded parameters and the single-process oracle forward for each case — TEST ONLY."""
from oracle import sage_ref
from truth_recommendation_gnn_amd import HeteroSAGE, WeightedRGCN, synth
from truth_recommendation_gnn_amd.parallel import RELATIONS

REL3 = [(synth.REV_ENGAGES, 1.0), (synth.SOCIAL, 0.75), (synth.ENGAGES, 1.0)]
REL4 = [(synth.REV_ENGAGES, 1.0), (synth.SOCIAL, 0.75), (synth.ENGAGES, 1.0),
        (synth.POST_POST, 0.5)]


def _param_shapes(cfg, relations=RELATIONS):
    out = []
    for l in range(cfg.layers):
        cin = cfg.dim if l == 0 else cfg.hidden
        for et, _ in relations:
            p = f"layers.{l}.{'__'.join(et)}"
            out += [(f"{p}.lin_l.weight", (cfg.hidden, cin)), (f"{p}.lin_l.bias", (cfg.hidden,)),
                    (f"{p}.lin_r.weight", (cfg.hidden, cin))]
    return out


def _rgcn_shapes(h, d):
    return [(f"{m}.{k}", (h, d) if k.endswith("weight") else (h,))
            for m in ("msg_direct", "msg_social", "post_update")
            for k in ("lin_l.weight", "lin_l.bias", "lin_r.weight")]


def _tiny(layers):
    """7 users / 3 posts split over 3 ranks (users [0,3) [3,6) [6,7), one post row each): the
    last rank owns no engages edge and no social in-edge, a duplicate edge and a self loop are
    kept, and one post slice receives no post->post edge."""
    import torch
    cfg = synth.GraphConfig("tiny", 7, 3, 7, 5, 3, 8, 8, layers)
    eng = torch.tensor([[0, 1, 1, 3, 4, 4, 5], [0, 0, 1, 2, 0, 0, 1]])
    soc = torch.tensor([[6, 2, 4, 0, 5], [0, 4, 4, 5, 1]])
    pp = torch.tensor([[1, 2, 0], [0, 0, 2]])
    gen = torch.Generator().manual_seed(5)
    x = {"user": torch.randn(7, 8, generator=gen), "post": torch.randn(3, 8, generator=gen)}
    e = {synth.ENGAGES: eng, synth.REV_ENGAGES: eng.flip(0), synth.SOCIAL: soc,
         synth.POST_POST: pp}
    return cfg, synth.SynthGraph(cfg, x, e)


def setup(kind):
    """(graph config, graph, model, params, oracle forward, edges handed to UserShard)."""
    if kind == "tiny_rgcn":
        cfg, g = _tiny(1)
        del g.edge_index_dict[synth.POST_POST]
        params = sage_ref.init_params(_rgcn_shapes(cfg.hidden, cfg.dim))
        model = WeightedRGCN(cfg.hidden)
        fwd = lambda P: sage_ref.weighted_rgcn(P, g.x_dict, g.edge_index_dict)
        return cfg, g, model, params, fwd, dict(g.edge_index_dict)
    if kind == "tiny4":
        cfg, g = _tiny(2)
        params = sage_ref.init_params(_param_shapes(cfg, REL4))
        model = HeteroSAGE(cfg.hidden, REL4, num_layers=cfg.layers)
        fwd = lambda P: sage_ref.hetero_sage(P, g.x_dict, g.edge_index_dict, REL4, cfg.layers)
        return cfg, g, model, params, fwd, dict(g.edge_index_dict)
    if kind == "engage2":
        cfg = synth.dataclasses.replace(synth.scaled("cfg2", 0.0005), dim=16, hidden=16)
        g = synth.make_graph(cfg)
        params = sage_ref.init_params(_param_shapes(cfg))
        model = HeteroSAGE(cfg.hidden, RELATIONS, num_layers=cfg.layers)
        fwd = lambda P: sage_ref.hetero_sage(P, g.x_dict, g.edge_index_dict, RELATIONS, cfg.layers)
        return cfg, g, model, params, fwd, g.edge_index_dict[synth.ENGAGES]
    if kind == "engage3":    # 3 layers: the sharded step pre-projects layers 2 and 3
        cfg = synth.dataclasses.replace(synth.scaled("cfg2", 0.0005), dim=16, hidden=16, layers=3)
        g = synth.make_graph(cfg)
        params = sage_ref.init_params(_param_shapes(cfg))
        model = HeteroSAGE(cfg.hidden, RELATIONS, num_layers=cfg.layers)
        fwd = lambda P: sage_ref.hetero_sage(P, g.x_dict, g.edge_index_dict, RELATIONS, cfg.layers)
        return cfg, g, model, params, fwd, g.edge_index_dict[synth.ENGAGES]
    if kind == "soc2":       # rev_engages + social -> user, engages -> post, 2 layers (halo +
        # pre-projection of rev_engages at layer 2)
        cfg = synth.dataclasses.replace(synth.scaled("cfg5", 0.0002), num_post_post=0,
                                        dim=16, hidden=16)
        g = synth.make_graph(cfg)
        edges = {et: g.edge_index_dict[et] for et, _ in REL3}
        params = sage_ref.init_params(_param_shapes(cfg, REL3))
        model = HeteroSAGE(cfg.hidden, REL3, num_layers=cfg.layers)
        fwd = lambda P: sage_ref.hetero_sage(P, g.x_dict, edges, REL3, cfg.layers)
        return cfg, g, model, params, fwd, edges
    if kind == "rgcn":       # the reference model: rev_engages + social -> user, engages -> post
        cfg = synth.dataclasses.replace(synth.scaled("cfg5", 0.0002), num_post_post=0,
                                        dim=16, hidden=16, layers=1)
        g = synth.make_graph(cfg)
        params = sage_ref.init_params(_rgcn_shapes(cfg.hidden, cfg.dim))
        model = WeightedRGCN(cfg.hidden)
        fwd = lambda P: sage_ref.weighted_rgcn(P, g.x_dict, g.edge_index_dict)
        return cfg, g, model, params, fwd, dict(g.edge_index_dict)
    cfg = synth.dataclasses.replace(synth.scaled("cfg5", 0.0002), dim=16, hidden=16)
    g = synth.make_graph(cfg)
    params = sage_ref.init_params(_param_shapes(cfg, REL4))
    model = HeteroSAGE(cfg.hidden, REL4, num_layers=cfg.layers)
    fwd = lambda P: sage_ref.hetero_sage(P, g.x_dict, g.edge_index_dict, REL4, cfg.layers)
    return cfg, g, model, params, fwd, dict(g.edge_index_dict)
