#!/usr/bin/env python3
"""cfg5 mini-batch throughput on one GPU: 9M users / 1M posts / 200M engages (+ reverse) / 90M
social / 10M post-post, d=h=128, fanout [15, 10], 1024 seed users + 1024 seed posts per batch:
sample -> 2-layer hetero SAGE forward on the blocks -> loss on the seed embeddings -> backward ->
Adam.  python scripts/sampler_bench.py [--scale 1.0] [--batches 20]

Under torch.distributed.run (N ranks, one GPU each; backend nccl = RCCL): data-parallel mini-batch
training as cfg5 names it for 8 GPUs — every rank holds the graph, samples its own seed slices
(rank r takes batches r, r+N, ... of the epoch's shuffled order), and the weight gradients are
summed with one all-reduce per batch (parallel.sync_grads).  Reports the whole job's batches/s
(max-over-ranks time) on rank 0."""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import HeteroSAGE, parallel, sampler, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--seeds", type=int, default=1024)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    cfg = synth.CONFIGS["cfg5"] if args.scale == 1.0 else synth.scaled("cfg5", args.scale)
    t0 = time.perf_counter()
    g = synth.make_graph(cfg, device=dev, device_gen=True)
    rels = [(synth.REV_ENGAGES, 1.0), (synth.SOCIAL, 0.75), (synth.ENGAGES, 1.0),
            (synth.POST_POST, 0.5)]
    num = {"user": cfg.num_users, "post": cfg.num_posts}
    s = sampler.NeighborSampler(num, g.edge_index_dict, [et for et, _ in rels], [15, 10])
    torch.cuda.synchronize()
    if rank == 0:
        print(f"graph + CSRs: {time.perf_counter() - t0:.1f} s", flush=True)
    torch.manual_seed(synth.WEIGHT_SEED)
    model = HeteroSAGE(cfg.hidden, rels, num_layers=2, in_channels=cfg.dim).to(dev)
    env = parallel.DistEnv.from_torch()
    if world > 1:                            # identical initial weights on every rank
        for prm in model.parameters():
            dist.broadcast(prm.data, 0)
    opt = None
    gen = torch.Generator(device=dev).manual_seed(0)
    stats = {"sample_ms": [], "step_ms": [], "edges": []}
    # one shuffle per epoch, as a loader over the seed nodes does; batches are slices of it
    order = {"user": torch.randperm(cfg.num_users, device=dev, generator=gen),
             "post": torch.randperm(cfg.num_posts, device=dev, generator=gen)}
    t_start = None
    for b in range(args.batches + 2):
        if b == 2:                               # timed region: batches 2 .. batches+1
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier(device_ids=[local])
            t_start = time.perf_counter()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gb = b * world + rank                    # this rank's slice of the epoch order
        seeds = {t: o[gb * args.seeds:(gb + 1) * args.seeds] for t, o in order.items()}
        mb = s.sample(seeds, seed=gb)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        out = sampler.forward_blocks(model, mb, g.x_dict)
        if opt is None:
            opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        # link loss on (seed user i, seed post i) pairs against shuffled posts as negatives
        u, p = out["user"], out["post"]
        pos = (u * p).sum(1)
        neg = (u * p.roll(1, 0)).sum(1)
        loss = torch.nn.functional.softplus(-pos).mean() + torch.nn.functional.softplus(neg).mean()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        parallel.sync_grads(model, env)          # no-op at world size 1
        opt.step()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if b >= 2:
            stats["sample_ms"].append((t1 - t0) * 1e3)
            stats["step_ms"].append((t2 - t1) * 1e3)
            stats["edges"].append(sum(blk.csr[et].num_edges for blk in mb.blocks for et in blk.csr))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(device_ids=[local])
    el = torch.tensor([time.perf_counter() - t_start], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    med = lambda v: sorted(v)[len(v) // 2]
    res = {"config": cfg.name, "n_gpus": world, "seeds_per_type": args.seeds, "fanouts": [15, 10],
           "sample_ms_median": round(med(stats["sample_ms"]), 3),
           "fwd_bwd_adam_ms_median": round(med(stats["step_ms"]), 3),
           "sampled_edges_per_batch_median": med(stats["edges"]),
           "batches_per_s": round(1e3 / (med(stats["sample_ms"]) + med(stats["step_ms"])), 1),
           "job_batches_per_s": round(world * args.batches / float(el), 1),
           "job_sampled_edges_per_s": round(world * sum(stats["edges"]) / float(el), 1)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
