"""Diagnostic: a cfg5 mini-batch (full size, or scaled by argv[1]); per layer and node type, the
HIP outputs and their gradients against plain torch on the same sampled blocks."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from oracle import sage_ref
from truth_recommendation_gnn_amd import HeteroSAGE, ops, sampler, synth
from truth_recommendation_gnn_amd.nn import _fused_weights
DEV = torch.device("cuda")
scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
cfg = synth.CONFIGS["cfg5"] if scale == 1.0 else synth.scaled("cfg5", scale)
g = synth.make_graph(cfg, device=DEV, device_gen=True)
rels = [(synth.REV_ENGAGES, 1.0), (synth.SOCIAL, 0.75), (synth.ENGAGES, 1.0), (synth.POST_POST, 0.5)]
num = {"user": cfg.num_users, "post": cfg.num_posts}
s = sampler.NeighborSampler(num, g.edge_index_dict, [et for et, _ in rels], [15, 10])
gen = torch.Generator(device=DEV).manual_seed(17)
nb = min(1024, cfg.num_posts)
seeds = {"user": torch.randperm(cfg.num_users, device=DEV, generator=gen)[:nb],
         "post": torch.randperm(cfg.num_posts, device=DEV, generator=gen)[:nb]}
mb = s.sample(seeds, seed=3)
for l, blk in enumerate(mb.blocks):
    print("block", l, {t: int(v.numel()) for t, v in mb.nodes[l].items()}, blk.n_dst,
          {et[1]: int(c.num_edges) for et, c in blk.csr.items()})
names = []
for l in range(cfg.layers):
    for et, _ in rels:
        p = f"layers.{l}.{'__'.join(et)}"
        names += [(f"{p}.lin_l.weight", (cfg.hidden, cfg.dim)), (f"{p}.lin_l.bias", (cfg.hidden,)),
                  (f"{p}.lin_r.weight", (cfg.hidden, cfg.dim))]
params = sage_ref.init_params(names)
model = HeteroSAGE(cfg.hidden, rels, num_layers=cfg.layers, in_channels=cfg.dim).to(DEV)
model.load_state_dict(params)

def run(hip):
    h = {t: g.x_dict[t][ids.long()] for t, ids in mb.nodes[0].items()}
    if not hip:
        h = {t: v.cpu() for t, v in h.items()}
        P = {k: v.clone().requires_grad_() for k, v in params.items()}
    outs = []
    for l, (convs, blk) in enumerate(zip(model.layers, mb.blocks)):
        out = {}
        for dst, n_dst in blk.n_dst.items():
            msgs = [("__".join(et), et, w) for et, w in rels if et[2] == dst and et in blk.csr]
            root = h[dst][:n_dst]
            if hip:
                W, b = _fused_weights(convs, msgs, h)
                aggrs = [ops.mean_gather(h[et[0]], blk.csr[et]) for _, et, _ in msgs]
                out[dst] = ops.fused_linear(aggrs + [root.contiguous()], W, b, True)
            else:
                acc = None
                for name, et, w in msgs:
                    wl, bl, wr = sage_ref._conv_params(P, f"layers.{l}.{name}")
                    m = sage_ref.sage_conv(h[et[0]], root, blk.csr[et].edge_index.cpu(), wl, bl, wr)
                    acc = w * m if acc is None else acc + w * m
                out[dst] = torch.relu(acc)
            out[dst].retain_grad()
        outs.append(out)
        h = out
    gg = torch.Generator().manual_seed(1)
    wts = {t: torch.randn(h[t].shape, generator=gg) for t in sorted(h)}
    loss = sum((h[t] * (wts[t].to(DEV) if hip else wts[t])).sum() for t in sorted(h))
    loss.backward()
    return outs

a, b = run(True), run(False)
for l in range(len(a)):
    for t in a[l]:
        x, y = a[l][t].detach().cpu(), b[l][t].detach()
        gx, gy = a[l][t].grad.cpu(), b[l][t].grad
        print(f"layer {l} {t}: out err {float((x-y).abs().max()):.3e} (max {float(y.abs().max()):.3e}); "
              f"grad err {float((gx-gy).abs().max()):.3e} (max {float(gy.abs().max()):.3e})")
        bad = ((gx - gy).abs() > 1e-4 * gy.abs().max()).any(1).nonzero().flatten()
        if bad.numel():
            print("   bad rows:", bad.numel(), bad[:10].tolist())
