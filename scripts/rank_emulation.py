#!/usr/bin/env python3
"""Per-rank compute of the weak-scaled N-GPU bench, on one GPU: a cfg2-sized user range (1M users,
20M engages) against the N x 100k post table every rank sees.  Runs the single-GPU fused step
(the post projection on all N x 100k posts, so it over-counts the sliced post side slightly);
collectives excluded.  python scripts/rank_emulation.py --world 8"""
import argparse
import dataclasses
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import HeteroSAGE, ops, synth  # noqa: E402
from truth_recommendation_gnn_amd.parallel import RELATIONS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda")
    base = synth.CONFIGS["cfg2"]
    cfg = dataclasses.replace(base, name=f"cfg2-rank-of-{args.world}",
                              num_posts=base.num_posts * args.world)
    g = synth.make_graph(cfg, device=dev, device_gen=True)
    pos = g.edge_index_dict[synth.ENGAGES]
    pw = synth.interaction_weights(cfg.num_posts).to(dev)[pos[1]]
    cscale = pw.mean()
    model = HeteroSAGE(cfg.hidden, RELATIONS, num_layers=cfg.layers).to(dev)
    with torch.no_grad():
        model(g.x_dict, g.edge_index_dict)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    gen = torch.Generator(device=dev).manual_seed(3)

    def step():
        opt.zero_grad(set_to_none=True)
        out = model(g.x_dict, g.edge_index_dict)
        neg = ops.sample_negatives(pos, cfg.num_posts, generator=gen)
        loss = ops.edge_bce_loss(out["user"], out["post"], pos, neg, pw, neg_order="user",
                                 check=False, cscale=cscale)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    timer = ops.KernelTimer()                 # one more pass for the per-kernel split
    ops.set_timer(timer)
    for _ in range(args.steps):
        step()
    ops.set_timer(None)
    kern = {k: round(v["ms"] / args.steps, 4) for k, v in sorted(timer.summary().items())}
    print(json.dumps({"world": args.world, "posts": cfg.num_posts,
                      "ms_per_step_compute": round(ms, 3), "kernels_ms_per_step": kern}))


if __name__ == "__main__":
    main()
