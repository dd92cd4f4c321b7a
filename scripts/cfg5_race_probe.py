#!/usr/bin/env python3
"""Does a cfg5 replay write outside its own memory?  The pipelined bench (the next batch staged on
a side stream under the replay) trains to a different loss than the same steps unpipelined
(round 6: 1.3075 vs 1.2959).  This builds the bench's captured step at full cfg5 scale, stages one
batch, then fills the STAGE arenas and the LinkSampler's scratch with a canary byte and replays the
graph (nothing else running): any canary byte that changes was written by the replay.
usage: python scripts/cfg5_race_probe.py [scale]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import HeteroSAGE, minibatch, sampler, synth  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda")
scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
cfg = synth.CONFIGS["cfg5"] if scale == 1.0 else synth.scaled("cfg5", scale)
g = synth.make_graph(cfg, device=dev, device_gen=True)
rels = bench.relations_of(cfg)
s = sampler.NeighborSampler({"user": cfg.num_users, "post": cfg.num_posts}, g.edge_index_dict,
                            [et for et, _ in rels], [15, 10])
torch.manual_seed(synth.WEIGHT_SEED)
model = HeteroSAGE(cfg.hidden, rels, num_layers=cfg.layers, in_channels=cfg.dim).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True, capturable=True)
pos_ei = g.edge_index_dict[synth.ENGAGES]
order = torch.randperm(int(pos_ei.shape[1]), device=dev,
                       generator=torch.Generator(device=dev).manual_seed(0), dtype=torch.int32)
B = 1024
ll = minibatch.LinkLoss(B, B, 2 * B, dev)
step = minibatch.CapturedStep(model, g.x_dict, s, {"user": B, "post": 2 * B}, ll, opt)
lb0 = minibatch.link_batch(pos_ei, order[:B].long(), cfg.num_posts)
lb0.mb = s.sample(lb0.seeds, seed=0)
ll.load(lb0.pu, lb0.pp, lb0.pn)
step.capture(lb0.mb, warmup=2)
ls = minibatch.LinkSampler(step, pos_ei, cfg.num_posts, ll)
gen = torch.Generator(device=dev).manual_seed(1)
ls.prepare(order[B:2 * B].long(), 1, gen)
step.step()
torch.cuda.synchronize()

regions = {"blocks.stage": step.blocks.arena._bytes["stage"],
           "loss.stage": ll.arena._bytes["stage"],
           "seeds.user": ls.seeds["user"], "seeds.post": ls.seeds["post"], "pairs": ls.pairs,
           "counts0": ls.counts[0], "counts1": ls.counts[1], "d_E": ls.d_E}
for h, hop in enumerate(ls._hops):
    if hop["items"] is not None:
        regions[f"items{h}"] = hop["items"]
    regions[f"hop_ws{h}"] = hop["ws"]
    if "rws" in hop:
        regions[f"relabel_ws{h}"] = hop["rws"]
# the same batch staged on a side stream and on the current one: equal bytes?
side = torch.cuda.Stream(dev)
snap = {}
for where in ("side", "main"):
    g2 = torch.Generator(device=dev).manual_seed(77)
    ids = order[3 * B:4 * B].long()
    torch.cuda.synchronize()
    if where == "side":
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            ls.prepare(ids, 3, g2)
    else:
        ls.prepare(ids, 3, g2)
    torch.cuda.synchronize()
    snap[where] = (step.blocks.arena._bytes["stage"].clone(), ll.arena._bytes["stage"].clone())
diff = {}
for name, (o, n, dt, nb) in step.blocks.arena.layout.items():
    m = int((snap["side"][0][o:o + nb] != snap["main"][0][o:o + nb]).sum())
    if m:
        diff["blocks." + name] = m
for name, (o, n, dt, nb) in ll.arena.layout.items():
    m = int((snap["side"][1][o:o + nb] != snap["main"][1][o:o + nb]).sum())
    if m:
        diff["loss." + name] = m
print({"stage side vs main, differing bytes": diff})
for k, t in regions.items():
    t.view(torch.uint8).fill_(0xA5)
torch.cuda.synchronize()
bad = {}
for rep in range(4):
    step.graph.replay()
    torch.cuda.synchronize()
    for k, t in regions.items():
        b = t.view(torch.uint8)
        n = int((b != 0xA5).sum())
        if n:
            idx = torch.nonzero(b != 0xA5).flatten()
            bad.setdefault(k, (n, int(idx[0]), int(idx[-1]), b.numel()))
print({"replays": 4, "changed": bad, "regions": list(regions)})
# where the stage arena's changed bytes fall in its layout
if "blocks.stage" in bad:
    b = step.blocks.arena._bytes["stage"]
    hit = torch.nonzero(b != 0xA5).flatten().cpu()
    for name, (o, n, dt, nb) in step.blocks.arena.layout.items():
        m = int(((hit >= o) & (hit < o + nb)).sum())
        if m:
            print("  blocks.stage", name, m, "of", nb)
