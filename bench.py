#!/usr/bin/env python3
"""Headline bench: edges/s (fwd+bwd) of hetero message passing on MI355X (BASELINE.json).

Workload (N=1): BASELINE config 2 — synthetic user<->post graph, 1M users / 100k posts / 20M
engages (+ the 20M reverse relation), d = h = 64, 2-layer relation-weighted SAGE
(``HeteroSAGE`` = the reference ``WeightedRGCN`` layer stacked twice).  One step = one training
step of ``train_gnn.py:242-285``: forward, the reference link loss over all 20M positive edges
with fresh ``torch.randint`` negatives, full backward, Adam.  Inputs resident in HBM before the
timed region.  Metric numerator = sum over layers and relations of E_r = 80M edges/step.

N>1 (``torch.distributed.run``): weak scaling — one global graph N times the cfg2 size (N·1M
users, N·100k posts, N·20M engages), destination-partitioned (parallel.py): each rank owns a
cfg2-sized user range and a 1/N row slice of the post table.  Per layer one RCCL reduce-scatter
of the post partial sums and one all-gather of the projected slices (their adjoints in the
backward), a halo all-to-all for user->user relations when the config has them (cfg5), weight
gradients all-reduced once per step.  The step is ``UserShard.step``: the same kernels as the
autograd path, with every collective issued as soon as its input is complete and awaited only
by its consumer (``--autograd-sharded`` runs forward + loss + backward() instead).
value = all ranks' edges / max-over-ranks time.

Prints ONE JSON line (rank 0) with ``roofline`` for the dominant kernel (the K1 forward gather:
algorithmic bytes per launch / HIP-event-timed duration inside the timed region) and
``cpu_baseline`` (the plain-torch CPU oracle on a bounded sample, rank 0 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from truth_recommendation_gnn_amd import HeteroSAGE, ops, synth  # noqa: E402
from truth_recommendation_gnn_amd import parallel  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured copy
FP32_MFMA_PEAK_TFS = 157.3  # same table: dense fp32 matrix (v_mfma_f32_16x16x4_f32), no xf32 on gfx950
# every relation a config may hold, with the reference's weights (train_gnn.py:163-164:
# w_direct 1.0, w_social 0.75); cfg5's post-post relation takes 1.0
ALL_RELATIONS = [(synth.REV_ENGAGES, 1.0), (synth.SOCIAL, 0.75), (synth.ENGAGES, 1.0),
                 (synth.POST_POST, 1.0)]


def relations_of(cfg):
    """The relations ``cfg``'s graph holds: cfg2-4 the two engage directions, cfg5 all four."""
    have = {synth.REV_ENGAGES, synth.ENGAGES}
    if cfg.num_social:
        have.add(synth.SOCIAL)
    if cfg.num_post_post:
        have.add(synth.POST_POST)
    return [(et, w) for et, w in ALL_RELATIONS if et in have]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="cfg2")
    p.add_argument("--scale", type=float, default=1.0, help="shrink the config (debug only)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--profile-steps", action="store_true",
                   help="no per-kernel events (for rocprofv3 runs)")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (= RCCL, the product path); gloo only to rehearse N>1 on one GPU")
    p.add_argument("--dist", action="store_true",
                   help="take the sharded path (process group + collectives) even at world size 1: "
                        "runs the RCCL calls on a 1-GPU box")
    p.add_argument("--autograd-sharded", action="store_true",
                   help="sharded path through autograd (forward + loss + backward()) instead of "
                        "UserShard.step's explicit collective schedule")
    p.add_argument("--strong", action="store_true",
                   help="N>1: partition the config's own graph over the ranks (strong scaling, e.g. "
                        "BASELINE cfg4 on 8 GPUs) instead of an N-times larger one")
    p.add_argument("--rccl-normal-priority", action="store_true",
                   help="RCCL collectives on a normal-priority stream (default: high priority)")
    p.add_argument("--same-device", action="store_true",
                   help="every rank on cuda:0 (rehearsal on a 1-GPU box, with --dist-backend gloo)")
    return p.parse_args()


def cpu_baseline(cfg, threads):
    """Oracle (plain torch CPU, PyG's op pattern) on a bounded cfg sample; edges/s."""
    from oracle import sage_ref
    torch.set_num_threads(threads)
    rels = relations_of(cfg)
    sample = synth.scaled(cfg.name, 0.05) if cfg.num_engages > 1_000_000 else cfg
    g = synth.make_graph(sample)
    names = []
    for l in range(sample.layers):
        cin = sample.dim if l == 0 else sample.hidden
        for et, _ in rels:
            p = f"layers.{l}.{'__'.join(et)}"
            names += [(f"{p}.lin_l.weight", (sample.hidden, cin)), (f"{p}.lin_l.bias", (sample.hidden,)),
                      (f"{p}.lin_r.weight", (sample.hidden, cin))]
    params = {k: v.requires_grad_() for k, v in sage_ref.init_params(names).items()}
    opt = torch.optim.Adam(params.values(), lr=1e-3)
    pos = g.edge_index_dict[synth.ENGAGES]
    pw = synth.interaction_weights(sample.num_posts)[pos[1]]

    def step():
        opt.zero_grad()
        out = sage_ref.hetero_sage(params, g.x_dict, g.edge_index_dict, rels, sample.layers)
        neg = torch.randint(0, sample.num_posts, (pos.shape[1],))
        loss = sage_ref.link_loss(out["user"], out["post"], pos, neg, pw)
        loss.backward()
        opt.step()

    step()
    t0 = time.perf_counter()
    n = 0
    while True:
        step()
        n += 1
        if time.perf_counter() - t0 > 10.0 or n >= 5:
            break
    dt = (time.perf_counter() - t0) / n
    edges = sample.layers * sum(int(g.edge_index_dict[et].shape[1]) for et, _ in rels)
    return {"value": edges / dt, "unit": "edges/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{sample.name}: U={sample.num_users} P={sample.num_posts} "
                      f"E_engage={sample.num_engages} d={sample.dim}, {sample.layers}-layer fwd+loss+"
                      f"bwd+Adam, mean of {n} steps after 1 warmup (oracle/sage_ref.py, torch CPU)"}


def _pg_options(args):
    """RCCL on a high-priority stream: every collective of the sharded step runs under compute
    kernels that fill the GPU, and the priority lets its workgroups be dispatched as soon as CUs
    free up instead of queueing behind the compute grid (``--rccl-normal-priority`` turns it
    off)."""
    if args.dist_backend != "nccl" or args.rccl_normal_priority:
        return None
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        return opts
    except (AttributeError, RuntimeError):
        return None


def _barrier(args, local):
    if args.dist_backend == "nccl":
        dist.barrier(device_ids=[local])
    else:
        dist.barrier()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    sharded = world > 1 or args.dist
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    if sharded:
        if "MASTER_ADDR" not in os.environ:          # plain `python bench.py --dist`
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29531", RANK="0",
                              WORLD_SIZE="1")
        dist.init_process_group(args.dist_backend, pg_options=_pg_options(args))
    dev = torch.device("cuda", local)
    cfg = synth.CONFIGS[args.config]
    if args.scale != 1.0:
        cfg = synth.scaled(args.config, args.scale)
    torch.manual_seed(synth.WEIGHT_SEED)
    gen = torch.Generator(device=dev).manual_seed(synth.NEG_SEED + rank)
    if not sharded:
        g = synth.make_graph(cfg, device=dev)
        pos = g.edge_index_dict[synth.ENGAGES]
        pw = synth.interaction_weights(cfg.num_posts).to(dev)[pos[1]]
        # BCEWithLogitsLoss() collapses the per-edge interaction weights to their mean
        # (train_gnn.py:276-281); the weights are static graph data, so the mean is taken once
        cscale = pw.mean()
        rels = relations_of(cfg)
        model = HeteroSAGE(cfg.hidden, rels, num_layers=cfg.layers).to(dev)
        with torch.no_grad():
            model(g.x_dict, g.edge_index_dict)  # materialise lazy weights, build + cache CSR/CSC
        edges_step = cfg.layers * sum(int(g.edge_index_dict[et].shape[1]) for et, _ in rels)

        def forward_loss():
            out = model(g.x_dict, g.edge_index_dict)
            neg = ops.sample_negatives(pos, cfg.num_posts, generator=gen)
            return ops.edge_bce_loss(out["user"], out["post"], pos, neg, pw, neg_order="user",
                                     check=False, cscale=cscale)
    else:
        env = parallel.DistEnv.from_torch()
        gcfg = cfg if (args.strong or args.scale != 1.0) else synth.replicated(args.config, world)
        g = synth.make_graph(gcfg, device=dev, device_gen=True)   # identical on every rank
        pos_g = g.edge_index_dict[synth.ENGAGES]
        pw_g = synth.interaction_weights(gcfg.num_posts).to(dev)[pos_g[1]]
        rels = relations_of(gcfg)
        shard = parallel.UserShard({et: g.edge_index_dict[et] for et, _ in rels}, gcfg.num_users,
                                   gcfg.num_posts, env, pos_weights=pw_g)
        x_user = g.x_dict["user"][shard.lo:shard.hi].contiguous()
        x_post = g.x_dict["post"]
        # global count over all relations
        edges_step = gcfg.layers * sum(int(g.edge_index_dict[et].shape[1]) for et, _ in rels)
        del g, pos_g, pw_g
        torch.cuda.empty_cache()
        model = HeteroSAGE(gcfg.hidden, rels, num_layers=gcfg.layers).to(dev)
        with torch.no_grad():
            shard.forward(model, x_user, x_post)
        for p in model.parameters():
            dist.broadcast(p.data, 0)
        cfg = gcfg

        def forward_loss():
            # the post table's last all-gather stays in flight under the negatives draw + sort
            h_u, h_p = shard.forward(model, x_user, x_post, wait=False)
            neg = ops.sample_negatives(shard.pos_local, gcfg.num_posts, generator=gen)
            return shard.loss(h_u, h_p, neg, neg_order="user")

    # the reference's optimizer (train_gnn.py:207, Adam lr 0.001) as torch's fused kernel: one
    # launch for every parameter instead of a multi-tensor chain per Adam stage
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)

    def step():
        opt.zero_grad(set_to_none=True)
        if sharded and not args.autograd_sharded:
            # explicit schedule: each collective issued when its input is complete and waited
            # for by its consumer only (parallel.UserShard.step; same kernels and gradients)
            neg = ops.sample_negatives(shard.pos_local, gcfg.num_posts, generator=gen)
            loss = shard.step(model, x_user, x_post, neg, neg_order="user")
        else:
            loss = forward_loss()
            loss.backward()
        if sharded:
            parallel.sync_grads(model, parallel.DistEnv.from_torch())
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    timer = None if args.profile_steps else ops.KernelTimer()
    torch.cuda.synchronize()
    if sharded:
        _barrier(args, local)
    ops.set_timer(timer)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if sharded:
        _barrier(args, local)
    t1 = time.perf_counter()
    ops.set_timer(None)
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if sharded:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed)
    value = edges_step * args.steps / elapsed     # edges_step is already the global count
    kern = timer.summary() if timer else {}
    if rank == 0:
        roof = None
        # Roofline kernel: K1 forward gather with the largest source table — the HBM-bound one
        # (user table, 256 MB at cfg2).  The post-table gathers (25.6 MB source) are served from
        # the 256 MB Infinity Cache and read above the HBM peak in algorithmic bytes; they are
        # listed under "kernels".
        # (sharded runs: the post partial sums are the weighted forward gathers, "gather_wfwd")
        fwd = {k: v for k, v in kern.items() if k.startswith(("gather_fwd", "gather_wfwd"))}
        if fwd:
            src_rows = lambda k: int(k.split("<-")[1].split("]")[0])
            name = max(fwd, key=src_rows)
            r = fwd[name]
            per_launch_ms = r["ms"] / r["launches"]
            per_launch_bytes = r["bytes"] / r["launches"]
            ach = per_launch_bytes / (per_launch_ms * 1e-3) / 1e9
            traffic, tsrc = None, None
            weighted = name.startswith("gather_wfwd")
            pmc = os.path.join(ROOT, "profiles", "pmc_gather_r1.json")
            # the PMC passes measured the unweighted K1 launch of the cfg2 single-GPU step
            if os.path.exists(pmc) and world == 1 and cfg.name == "cfg2" and not weighted:
                with open(pmc) as f:
                    pm = json.load(f)
                traffic, tsrc = pm.get("hbm_bytes_per_launch"), "profiles/pmc_gather_r1.json"
            roof = {"bound": "hbm",
                    "kernel": (f"k_gather K1 weighted fwd (post partial sums) {name}" if weighted
                               else f"k_gather K1 mean fwd {name}"),
                    "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "traffic_source": tsrc, "avg_launch_us": round(per_launch_ms * 1e3, 1),
                    "algorithmic_bytes_per_launch": int(per_launch_bytes),
                    "bytes_formula": ("4*E*(2+d) + 4*(N_dst+1) + 4*N_dst*d" if weighted
                                      else "4*E*(1+d) + 4*(N_dst+1) + 4*N_dst*d")}
        # The dense projection (K3) against the fp32 MFMA peak: the largest forward launch (the
        # user side), HIP-event timed like the gather; the PMC MFMA-busy fraction of the same
        # kernel comes from profiles/pmc_k3_r1.json (scripts/pmc_k3.sh) for cfg2.
        proj = None
        lin = {k: v for k, v in kern.items() if k.startswith("linear_fwd[") and v["flops"]}
        if lin:
            name = max(lin, key=lambda k: lin[k]["flops"] / lin[k]["launches"])
            r = lin[name]
            tfs = r["flops"] / (r["ms"] * 1e-3) / 1e12
            busy, bsrc = None, None
            pk = os.path.join(ROOT, "profiles", "pmc_k3_r1.json")
            if os.path.exists(pk) and cfg.name == "cfg2" and cfg.hidden == 64:
                with open(pk) as f:
                    busy = json.load(f)["kernels"].get("hgnn::k_linear_fwd_v4<64, 128>", {}).get(
                        "mfma_util")
                bsrc = "profiles/pmc_k3_r1.json"
            proj = {"bound": "mfma", "kernel": f"k_linear_fwd_v4 K3 {name}",
                    "achieved": round(tfs, 1), "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                    "frac": round(tfs / FP32_MFMA_PEAK_TFS, 4),
                    "hbm_GB/s": round(r["bytes"] / (r["ms"] * 1e-3) / 1e9, 1),
                    "avg_launch_us": round(r["ms"] / r["launches"] * 1e3, 1),
                    "flops_per_launch": int(r["flops"] / r["launches"]),
                    "flops_formula": "2*N*K*H (K = sum of the input segments)",
                    "mfma_busy_pmc": busy, "mfma_busy_source": bsrc}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(cfg, args.cpu_threads)
        line = {
            "metric": "edges/s (fwd+bwd) hetero message-passing",
            "value": round(value, 1), "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong" if args.strong else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded numpy PCG64 graph, Zipf post degrees; random-init weights)",
            "config": {"workload": f"{cfg.name}: U={cfg.num_users} P={cfg.num_posts} "
                                   f"E_engage={cfg.num_engages} (+reverse), "
                                   f"relations={'+'.join(et[1] for et, _ in relations_of(cfg))}, "
                                   f"d=h={cfg.dim}, "
                                   f"{cfg.layers}-layer hetero-SAGE train step (fwd+loss+bwd+Adam)",
                       "edges_per_step": edges_step, "global_batch": edges_step,
                       "parallelism": (f"user-shard x{world} (post-table slices: RCCL "
                                       "reduce-scatter / all-gather per layer)"
                                       if sharded else "single")},
            "roofline": roof, "projection": proj, "cpu_baseline": cpu,
            "kernels": {k: {"launches": v["launches"], "ms_per_step": round(v["ms"] / args.steps, 4),
                            "GB/s": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] else None,
                            "compulsory_GB/s": (round(v["cbytes"] / (v["ms"] * 1e-3) / 1e9, 1)
                                                if v["ms"] else None),
                            **({"TFLOP/s": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1)}
                               if v["flops"] and v["ms"] else {})}
                        for k, v in sorted(kern.items())},
            "loss": float(loss.detach()),
        }
        print(json.dumps(line), flush=True)
    if sharded:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
