#!/usr/bin/env python3
"""Headline bench: edges/s (fwd+bwd) of hetero message passing on MI355X (BASELINE.json).

Workload — BASELINE ``configs[3]``, the graph the north_star's targets are stated on (cfg4):
synthetic 9M users / 1M posts (10M nodes) / 200M engages + the 200M reverse relation, d = h =
128, 2-layer relation-weighted SAGE (``HeteroSAGE`` = the reference ``WeightedRGCN`` layer
stacked twice).  One step = one training step of ``train_gnn.py:242-285``: forward, the
reference link loss over all 200M positive edges with fresh ``torch.randint``-distributed
negatives, full backward, Adam.  Inputs are resident in HBM before the timed region.  Metric
numerator = sum over layers and relations of E_r = 800M edges/step.

* ``--gpus 1`` (default): the whole cfg4 graph on one MI355X (it fits: ~60 GB resident).
* ``--gpus N`` (N > 1): STRONG scaling of the same cfg4 graph, destination-partitioned over N
  ranks (``parallel.UserShard``): each rank owns 1/N of the users and a 1/N row slice of the post
  table; per layer one RCCL reduce-scatter of the post partial sums and one all-gather of the
  projected slices (their adjoints in the backward); weight gradients all-reduced once per step.
  ``--weak`` instead grows the graph N-fold (each rank a cfg-sized share).
  Launch: under ``torch.distributed.run`` (RANK/WORLD_SIZE in the environment) every process is
  one rank; run as plain ``python bench.py --gpus N`` the script starts the N rank processes
  itself (spawned interpreters, before this process touches the GPU) and exits with their
  status.  A world size that disagrees with ``--gpus`` is an error, never a silent 1-GPU run.
* ``--config cfg2|cfg3`` (1 GPU): the smaller BASELINE configs; ``--config cfg5``: the
  4-relation neighbour-sampled mini-batch workload (``sampler.py``; one step = one mini-batch per
  rank, data-parallel over N ranks).

value = all ranks' edges / max-over-ranks wall time of exactly ``--steps`` steps, bracketed by a
barrier + device synchronise, with NO per-kernel events inside.  A second, separately timed run
of ``--timer-steps`` steps records HIP events around every kernel (on the stream it is launched
on) for ``roofline`` — the dominant HBM kernel, the K1 forward gather over the largest source
table: algorithmic bytes per launch / average launch time, ``traffic`` from the committed PMC
passes of the same launch (the newest ``profiles/pmc_r*.json``) — and for ``projection`` (K3 vs the fp32
MFMA peak).  ``cpu_baseline`` (rank 0, N=1 only): the plain-torch CPU oracle (PyG's op pattern)
on the box's allotted host cores, median of 5 steps after 2 warm-ups, on a stated down-scaled
sample of the same graph family (same degree distributions, so per-edge work is the same).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from truth_recommendation_gnn_amd import HeteroSAGE, synth  # noqa: E402
from truth_recommendation_gnn_amd import optim, parallel  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured copy
FP32_MFMA_PEAK_TFS = 157.3  # same table: dense fp32 matrix (v_mfma_f32_16x16x4_f32), no xf32 on gfx950
BF16_MFMA_PEAK_TFS = 2500.0  # same table: dense bf16 matrix (~2.5 PF; the 5 PF figure is 2:1 sparse)
DEFAULT_CONFIG = "cfg4"
# every relation a config may hold, with the reference's weights (train_gnn.py:163-164:
# w_direct 1.0, w_social 0.75); cfg5's post-post relation takes 1.0
ALL_RELATIONS = [(synth.REV_ENGAGES, 1.0), (synth.SOCIAL, 0.75), (synth.ENGAGES, 1.0),
                 (synth.POST_POST, 1.0)]
# CPU-baseline sample: the config scaled by this factor (≈5 s per CPU step on 8 container cores,
# so 7 steps stay within the bench's few-minute budget)
CPU_SAMPLE_SCALE = {"cfg1": 1.0, "cfg2": 1 / 16, "cfg3": 1 / 16, "cfg4": 1 / 128, "cfg5": 1 / 128}


def relations_of(cfg):
    """The relations ``cfg``'s graph holds: cfg2-4 the two engage directions, cfg5 all four."""
    have = {synth.REV_ENGAGES, synth.ENGAGES}
    if cfg.num_social:
        have.add(synth.SOCIAL)
    if cfg.num_post_post:
        have.add(synth.POST_POST)
    return [(et, w) for et, w in ALL_RELATIONS if et in have]


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default=DEFAULT_CONFIG)
    p.add_argument("--weak", action="store_true",
                   help="N>1: an N-times larger graph, each rank a config-sized share (default: "
                        "strong scaling, the config's own graph split N ways)")
    p.add_argument("--strong", action="store_true", help="(the default at N>1; kept for old "
                   "command lines)")
    p.add_argument("--full-batch", action="store_true",
                   help="cfg5: the full-graph 4-relation step instead of the sampled mini-batches")
    p.add_argument("--batch-seeds", type=int, default=1024,
                   help="cfg5 mini-batch: positive engages edges per batch per rank (one uniform "
                        "negative post each; the seeds are their distinct endpoints)")
    p.add_argument("--torch-loss", action="store_true",
                   help="cfg5 mini-batch: the link loss as torch ops instead of the fused kernels")
    p.add_argument("--no-graph", action="store_true",
                   help="cfg5 mini-batch: run the step eagerly instead of replaying its HIP graph")
    p.add_argument("--eager-allreduce", action="store_true",
                   help="cfg5 mini-batch over RCCL: the gradient all-reduce eagerly between two "
                        "graph replays instead of recorded inside the one graph")
    p.add_argument("--no-prefetch", action="store_true",
                   help="cfg5 mini-batch: no side-stream sampling of the next batch")
    p.add_argument("--prefetch", action="store_true",
                   help="cfg5 mini-batch: sample the next batch on a side stream under this one")
    p.add_argument("--single-buffer", action="store_true",
                   help="cfg5 mini-batch: one recorded step, each batch staged and copied into "
                        "its buffers, instead of two steps over their own buffers in turn")
    p.add_argument("--side-cus", type=int, default=0,
                   help="cfg5 mini-batch: run the side stream's sampling on this many CUs only "
                        "(a CU-masked stream; 0: all)")
    p.add_argument("--default-priority", action="store_true",
                   help="cfg5 mini-batch: replay on a default-priority stream (by default the "
                        "steps run on a high-priority one, above the side stream's sampling)")
    p.add_argument("--native-adam", action="store_true",
                   help="optim.Adam (one native launch over every parameter) instead of "
                        "torch.optim.Adam(fused=True)")
    p.add_argument("--eager-sampler", action="store_true",
                   help="cfg5 mini-batch: sample with the eager NeighborSampler (host-sized "
                        "launches, read-backs) and stage its batches, instead of the sync-free "
                        "LinkSampler")
    p.add_argument("--scale", type=float, default=1.0, help="shrink the config (debug only)")
    p.add_argument("--timer-steps", type=int, default=5,
                   help="steps of the separate per-kernel-event run (0: none)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=None,
                   help="default: the box's allotted CPUs (OMP_NUM_THREADS / affinity)")
    p.add_argument("--cpu-sample-scale", type=float, default=None,
                   help="cfg5: the CPU baseline's down-scaled sample")
    p.add_argument("--cpu-steps", type=int, default=3,
                   help="timed CPU-baseline steps of the full-batch configs (median, after one "
                        "warm-up; cfg4's 1/8 shard takes ~60 s a step on 16 cores)")
    p.add_argument("--cpu-shard", type=int, default=None,
                   help="full-batch configs: time rank 0's 1/S destination shard on the CPU oracle "
                        "(default: cfg4 8, cfg2/cfg3 1 = the whole graph)")
    p.add_argument("--no-presort-negatives", action="store_true",
                   help="N = 1: group the loss's negatives inside the loss, not on a side stream "
                        "under the forward (A/B: 154.9 / 155.0 vs 153.9 / 154.4 ms with it)")
    p.add_argument("--profile-steps", action="store_true",
                   help="no per-kernel-event run (for rocprofv3 runs)")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (= RCCL, the product path); gloo only to rehearse N>1 on one GPU")
    p.add_argument("--dist", action="store_true",
                   help="take the sharded path (process group + collectives) even at world size 1")
    p.add_argument("--autograd-sharded", action="store_true",
                   help="sharded path through autograd (forward + loss + backward()) instead of "
                        "UserShard.step's explicit collective schedule")
    p.add_argument("--dist-timeout", type=float, default=300.0,
                   help="seconds a collective may wait before the process group aborts the job "
                        "(a rank that issues another collective schedule fails within minutes, "
                        "not after the default 10; graph setup runs before the first collective "
                        "on every rank alike)")
    p.add_argument("--rccl-normal-priority", action="store_true",
                   help="RCCL collectives on a normal-priority stream (default: high priority)")
    p.add_argument("--same-device", action="store_true",
                   help="every rank on cuda:0 (rehearsal on a 1-GPU box, with --dist-backend gloo)")
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu: rehearse the launcher and sharded schedule on host cores with the "
                        "compute ops a test injects (tests/test_bench_launch.py); never a "
                        "measurement")
    p.add_argument("--json-out", default=None, help="also write the JSON line to this file")
    return p.parse_args(argv)


# ----------------------------------------------------------------------------- CPU baseline
def host_cores():
    """(physical cores of the host from lscpu, CPUs allotted to this job)."""
    phys = None
    try:
        out = subprocess.run(["lscpu", "-p=CORE,SOCKET"], capture_output=True, text=True,
                             timeout=10).stdout
        phys = len({ln for ln in out.splitlines() if ln and not ln.startswith("#")}) or None
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        allotted = len(os.sched_getaffinity(0))
    except AttributeError:
        allotted = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        allotted = min(allotted, int(omp))
    if phys:
        allotted = min(allotted, phys)
    return phys, allotted


def cpu_baseline(cfg, threads=None, scale=None):
    """The plain-torch CPU oracle (PyG's op pattern: materialised ``index_select``,
    ``scatter_reduce`` mean, ``addmm``) running the same training step on a down-scaled graph of
    the same family; edges/s = median over 5 steps after 2 warm-ups.  (The cfg5 mini-batch
    line's comparison; the full-batch lines use :func:`cpu_baseline_shard`.)"""
    from oracle import sage_ref
    phys, allotted = host_cores()
    threads = threads or allotted
    torch.set_num_threads(threads)
    rels = relations_of(cfg)
    f = scale if scale is not None else CPU_SAMPLE_SCALE.get(cfg.name.split("x")[0], 1 / 64)
    sample = cfg if f >= 1.0 else synth.dataclasses.replace(
        synth.scaled(cfg.name.split("x")[0], f), dim=cfg.dim, hidden=cfg.hidden,
        layers=cfg.layers)
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

    for _ in range(2):
        step()
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    dt = statistics.median(times)
    edges = sample.layers * sum(int(g.edge_index_dict[et].shape[1]) for et, _ in rels)
    return {"value": round(edges / dt, 1), "unit": "edges/s", "cores": threads,
            "host_physical_cores": phys, "kind": "port",
            "sample": f"{cfg.name} family scaled x{f:g}: U={sample.num_users} "
                      f"P={sample.num_posts} E_engage={sample.num_engages} d=h={sample.dim}, "
                      f"{sample.layers}-layer fwd+loss+bwd+Adam ({edges} edges/step); median of "
                      f"5 steps after 2 warm-ups ({dt:.2f} s/step), oracle/sage_ref.py on torch "
                      f"CPU with {threads} threads = the CPUs allotted to this job "
                      f"(host has {phys} physical cores); edges/s extrapolates linearly "
                      f"(per-edge work is scale-free, the sample's smaller tables favour the CPU)"}


def cpu_baseline_sampled(lb, x_dict, rels, cfg, threads=None, steps=5, warmup=1):
    """The cfg5 line's CPU baseline on the SAME sampled workload: one link
    mini-batch's blocks as the GPU step ran them, copied to the host (the input rows of its
    outermost block, each block's relations as local COO edge lists), then the oracle's step on
    them — ``oracle/sage_ref.py``'s PyG op pattern per block (materialised ``index_select``,
    ``scatter_reduce`` mean, ``addmm``; ``hetero_sage_blocks``), the reference's BCE link loss
    over the batch's positive and negative pairs (``link_loss``, unit edge weights as the GPU
    line's), backward, Adam.  edges/s = the batch's sampled message edges / the median step."""
    from oracle import sage_ref
    phys, allotted = host_cores()
    threads = threads or allotted
    torch.set_num_threads(threads)
    mb = lb.mb
    x_in = {t: x_dict[t].index_select(0, ids.long()).cpu() for t, ids in mb.nodes[0].items()}
    blocks, n_edges = [], 0
    for blk in mb.blocks:
        eid = {}
        for et, csr in blk.csr.items():
            rp, col = csr.fwd.rowptr.long().cpu(), csr.fwd.col.long().cpu()
            dst = torch.repeat_interleave(torch.arange(rp.numel() - 1), rp[1:] - rp[:-1])
            eid[et] = torch.stack([col[:dst.numel()], dst])
            n_edges += int(dst.numel())
        blocks.append((eid, dict(blk.n_dst)))
    names = []
    for l in range(cfg.layers):
        cin = cfg.dim if l == 0 else cfg.hidden
        for et, _ in rels:
            p = f"layers.{l}.{'__'.join(et)}"
            names += [(f"{p}.lin_l.weight", (cfg.hidden, cin)), (f"{p}.lin_l.bias", (cfg.hidden,)),
                      (f"{p}.lin_r.weight", (cfg.hidden, cin))]
    params = {k: v.requires_grad_() for k, v in sage_ref.init_params(names).items()}
    opt = torch.optim.Adam(params.values(), lr=1e-3)
    pos = torch.stack([lb.pu.long().cpu(), lb.pp.long().cpu()])
    neg = lb.pn.long().cpu()
    ones = torch.ones(pos.shape[1])

    def step():
        opt.zero_grad()
        out = sage_ref.hetero_sage_blocks(params, x_in, blocks, rels)
        loss = sage_ref.link_loss(out["user"], out["post"], pos, neg, ones)
        loss.backward()
        opt.step()

    for _ in range(warmup):
        step()
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    dt = statistics.median(times)
    return {"value": round(n_edges / dt, 1), "unit": "edges/s", "cores": threads,
            "host_physical_cores": phys, "kind": "port",
            "sample": (f"one sampled link mini-batch of the GPU line (the sampled blocks: "
                       f"{', '.join(str(sum(1 for _ in b[0])) + ' relations' for b in blocks)}, "
                       f"{n_edges} message edges, {pos.shape[1]} positive + {neg.numel()} negative "
                       f"pairs, input rows {', '.join(f'{t} {v.shape[0]}' for t, v in x_in.items())}"
                       f"), copied to the host: oracle/sage_ref.py hetero_sage_blocks + link_loss "
                       f"+ backward + Adam, d=h={cfg.dim}; median of {steps} steps after "
                       f"{warmup} warm-up ({dt * 1e3:.1f} ms/step), {threads} threads = the CPUs "
                       f"allotted to this job (host has {phys} physical cores)")}


# SURVEY §8d's CPU baseline for the full-batch configs: cfg2 / cfg3 whole, cfg4 (which needs
# >100 GB per materialised [E, d] relation on the oracle) as a destination shard: the 1/8 shard
# SURVEY §8d names (rank 0 of the 8-GPU split), the median of 3 timed steps after one warm-up,
# ~4 minutes of the bench's wall time on 16 cores.
CPU_SHARD = {"cfg4": 8}


def cpu_baseline_shard(cfg, g, rels, threads=None, shard=None, steps=3, warmup=1):
    """The oracle's training step (oracle/sage_ref.py: PyG's op pattern, materialised
    ``index_select`` + ``scatter_reduce`` mean + ``addmm``; train_gnn.py:242-285) over rank 0's
    DESTINATION SHARD of the graph the GPU line timed, at ``shard`` ranks: users [0, U/S) and post
    rows [0, P/S) are the destinations, each with ALL of its in-edges (rev_engages into the users,
    engages into the posts), read from the full 9M / 1M-row source tables; rows a shard does not
    own stand in for the tables the other ranks would provide (values irrelevant to the timing).
    The loss is the reference's over the shard users' positive edges.  2 layers fwd + loss + bwd
    + Adam; edges/s = the shard's edges per step (layers x in-edges of its destinations) / the
    median step time, which is the whole graph's rate when the S shards run one after another on
    these cores.  S = 1 is the whole graph (cfg2, cfg3)."""
    from oracle import sage_ref
    import torch.nn.functional as F
    phys, allotted = host_cores()
    threads = threads or allotted
    torch.set_num_threads(threads)
    S = shard if shard is not None else CPU_SHARD.get(cfg.name.split("x")[0], 1)
    U, P = cfg.num_users, cfg.num_posts
    nu, npo = -(-U // S), -(-P // S)
    e = g.edge_index_dict[synth.ENGAGES]
    # the shard's edges, selected where the graph lives, then moved to the host
    m_u = e[0] < nu                                  # rev_engages into own users
    m_p = e[1] < npo                                 # engages into own posts
    rev = torch.stack([e[1][m_u], e[0][m_u]]).cpu()  # (post -> own user)
    eng = torch.stack([e[0][m_p], e[1][m_p]]).cpu()  # (user -> own post)
    pw = synth.interaction_weights(P)[rev[0]]        # the own users' positive edges
    x_user, x_post = g.x_dict["user"].cpu(), g.x_dict["post"].cpu()
    names = []
    for l in range(cfg.layers):
        cin = cfg.dim if l == 0 else cfg.hidden
        for et, _ in rels:
            p = f"layers.{l}.{'__'.join(et)}"
            names += [(f"{p}.lin_l.weight", (cfg.hidden, cin)), (f"{p}.lin_l.bias", (cfg.hidden,)),
                      (f"{p}.lin_r.weight", (cfg.hidden, cin))]
    params = {k: v.requires_grad_() for k, v in sage_ref.init_params(names).items()}
    opt = torch.optim.Adam(params.values(), lr=1e-3)
    ru, rp = "__".join(synth.REV_ENGAGES), "__".join(synth.ENGAGES)
    own_u, own_p = torch.arange(nu), torch.arange(npo)
    pos = torch.stack([rev[1], rev[0]])              # (own user, post)
    gen = torch.Generator().manual_seed(synth.NEG_SEED)

    def conv(l, rel, x_src, x_dst, ei):
        return sage_ref.sage_conv(x_src, x_dst, ei, *sage_ref._conv_params(params, f"layers.{l}.{rel}"))

    def step():
        opt.zero_grad()
        tab_u, tab_p = x_user, x_post
        h_u, h_p = x_user[:nu], x_post[:npo]
        for l in range(cfg.layers):
            h_u = F.relu(conv(l, ru, tab_p, h_u, rev))
            h_p = F.relu(conv(l, rp, tab_u, h_p, eng))
            # the next layer's source tables: the shard's own rows, the rest stand-ins
            tab_u = x_user.index_copy(0, own_u, h_u)
            tab_p = x_post.index_copy(0, own_p, h_p)
        neg = torch.randint(0, P, (pos.shape[1],), generator=gen)
        loss = sage_ref.link_loss(h_u, tab_p, pos, neg, pw)
        loss.backward()
        opt.step()

    for _ in range(warmup):
        t0 = time.perf_counter()
        step()
        print(f"cpu_baseline: warm-up step {time.perf_counter() - t0:.1f} s", file=sys.stderr,
              flush=True)
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
        print(f"cpu_baseline: step {times[-1]:.1f} s", file=sys.stderr, flush=True)
    dt = statistics.median(times)
    edges = cfg.layers * (int(rev.shape[1]) + int(eng.shape[1]))
    total = cfg.layers * 2 * int(e.shape[1])
    return {"value": round(edges / dt, 1), "unit": "edges/s", "cores": threads,
            "host_physical_cores": phys, "kind": "port",
            "sample": (f"{cfg.name}: " + ("the whole graph" if S == 1 else
                       f"rank 0's 1/{S} destination shard (users [0,{nu}), post rows [0,{npo}) "
                       f"with all their in-edges: {int(rev.shape[1])} rev_engages + "
                       f"{int(eng.shape[1])} engages, full {U}/{P}-row source tables)")
                       + f", d=h={cfg.dim}, {cfg.layers}-layer fwd+loss+bwd+Adam, {edges} edges/step"
                       + ("" if S == 1 else f" ({edges / total:.4f} of the graph's {total}; "
                          f"x{S} extrapolation: the whole step ~{dt * S:.0f} s on these cores)")
                       + f"; median of {steps} steps after {warmup} warm-up ({dt:.2f} s/step), "
                       f"oracle/sage_ref.py op pattern on torch CPU, {threads} threads = the CPUs "
                       f"allotted to this job (host has {phys} physical cores)")}


# ----------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_entry(local_rank, world, port, argv, impl_factory):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    run(parse(argv), impl=impl_factory() if impl_factory is not None else None)


def launch(argv, impl_factory=None):
    """Start ``--gpus`` rank processes of this bench (fresh interpreters: nothing here has
    touched the GPU) and wait for them; a failing rank fails the launch."""
    import torch.multiprocessing as mp
    args = parse(argv)
    mp.start_processes(_rank_entry, args=(args.gpus, _free_port(), argv, impl_factory),
                       nprocs=args.gpus, join=True, start_method="spawn")


def main(argv=None, impl_factory=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            launch(argv, impl_factory)
            return
    elif int(env_world) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}; "
                         "refusing to report a world size the run does not use")
    run(args, impl=impl_factory() if impl_factory is not None else None)


# ----------------------------------------------------------------------------- one rank
def _pg_options(args):
    """RCCL on a high-priority stream: every collective of the sharded step runs under compute
    kernels that fill the GPU, and the priority lets its workgroups be dispatched as soon as CUs
    free up instead of queueing behind the compute grid (``--rccl-normal-priority`` turns it
    off)."""
    if args.dist_backend != "nccl" or args.rccl_normal_priority or args.device == "cpu":
        return None
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        return opts
    except (AttributeError, RuntimeError):
        return None


def _pmc_file():
    """The newest committed PMC summary (profiles/pmc_r<round>.json, scripts/pmc_r2.sh)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_r[0-9]*.json")),
                   key=lambda f: int("".join(ch for ch in os.path.basename(f) if ch.isdigit())))
    return files[-1] if files else None


def _pmc_traffic(cfg_name, world, kernel):
    """Per-launch HBM bytes of ``kernel`` from the committed PMC passes (scripts/pmc_r2.sh ->
    profiles/pmc_r<round>.json), for the same config and world size; (None, None) if absent."""
    path = _pmc_file()
    if path is None:
        return None, None
    with open(path) as f:
        pm = json.load(f)
    rec = pm.get("launches", {}).get(f"{cfg_name}|n{world}|{kernel}")
    if not rec:
        return None, None
    return (rec.get("hbm_bytes_per_launch"),
            f"profiles/{os.path.basename(path)} ({rec.get('source', '')})")


def _pmc_ratio(cfg_name, world, kernel):
    """PMC HBM bytes / algorithmic bytes of ``kernel`` (the newest profiles/pmc_r*.json)."""
    path = _pmc_file()
    if path is None:
        return None
    with open(path) as f:
        rec = json.load(f).get("launches", {}).get(f"{cfg_name}|n{world}|{kernel}")
    return rec.get("traffic_over_algorithmic") if rec else None


def _workload_config(args, world):
    cfg = synth.CONFIGS[args.config]
    if args.scale != 1.0:
        cfg = synth.scaled(args.config, args.scale)
    if world > 1 and args.weak:
        cfg = synth.replicated(args.config, world) if args.scale == 1.0 else \
            synth.dataclasses.replace(
                cfg, name=f"{cfg.name}x{world}gpu", num_users=cfg.num_users * world,
                num_posts=cfg.num_posts * world, num_engages=cfg.num_engages * world,
                num_social=cfg.num_social * world, num_post_post=cfg.num_post_post * world)
    return cfg


class _Clock:
    """Barrier + device synchronise on both sides; max over ranks."""

    def __init__(self, dev, sharded, args, local):
        self.dev, self.sharded, self.args, self.local = dev, sharded, args, local

    def sync(self):
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)
        if self.sharded:
            if self.args.dist_backend == "nccl" and self.dev.type == "cuda":
                dist.barrier(device_ids=[self.local])
            else:
                dist.barrier()

    def time(self, fn, n):
        self.sync()
        t0 = time.perf_counter()
        out = None
        for _ in range(n):
            out = fn()
        self.sync()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=self.dev)
        if self.sharded:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el), out


def run(args, impl=None):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    on_cpu = args.device == "cpu"
    if on_cpu and impl is None:
        raise SystemExit("bench.py --device cpu is a launcher rehearsal: the compute ops must be "
                         "injected (tests/test_bench_launch.py); there is no CPU product path")
    sharded = world > 1 or args.dist or on_cpu
    if args.same_device:
        local = 0
    if not on_cpu:
        torch.cuda.set_device(local)
    if sharded:
        if "MASTER_ADDR" not in os.environ:          # plain `python bench.py --dist`
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
                              RANK="0", WORLD_SIZE="1")
        # a mismatched collective schedule (tests/test_collective_schedule.py guards against
        # one) must fail inside the driver's time limit: bounded timeout, and RCCL's watchdog
        # tears the process group down on it instead of leaving the ranks blocked
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        import datetime
        dist.init_process_group("gloo" if on_cpu else args.dist_backend,
                                timeout=datetime.timedelta(seconds=args.dist_timeout),
                                pg_options=_pg_options(args))
    dev = torch.device("cpu") if on_cpu else torch.device("cuda", local)
    try:
        if args.config == "cfg5" and not args.full_batch:
            line = _run_minibatch(args, dev, world, rank, local, sharded, impl)
        else:
            line = _run_full_batch(args, dev, world, rank, local, sharded, impl)
        if rank == 0:
            s = json.dumps(line)
            print(s, flush=True)
            if args.json_out:
                with open(args.json_out, "w") as f:
                    f.write(s + "\n")
    finally:
        if sharded:
            dist.destroy_process_group()


def _run_full_batch(args, dev, world, rank, local, sharded, impl):
    from truth_recommendation_gnn_amd import ops
    on_cpu = dev.type == "cpu"
    cfg = _workload_config(args, world)
    torch.manual_seed(synth.WEIGHT_SEED)
    gen = torch.Generator(device=dev).manual_seed(synth.NEG_SEED + rank)
    rels = relations_of(cfg)
    t_setup = time.perf_counter()
    if not sharded:
        g = synth.make_graph(cfg, device=dev, device_gen=True)   # the graph the shards hold
        pos = g.edge_index_dict[synth.ENGAGES]
        pw = synth.interaction_weights(cfg.num_posts).to(dev)[pos[1]]
        # BCEWithLogitsLoss() collapses the per-edge interaction weights to their mean
        # (train_gnn.py:276-281); the weights are static graph data, so the mean is taken once
        cscale = pw.mean()
        model = HeteroSAGE(cfg.hidden, rels, num_layers=cfg.layers, in_channels=cfg.dim).to(dev)
        with torch.no_grad():
            model(g.x_dict, g.edge_index_dict)  # build + cache the CSR/CSC of every relation
        edges_step = cfg.layers * sum(int(g.edge_index_dict[et].shape[1]) for et, _ in rels)

        side = torch.cuda.Stream(dev) if not args.no_presort_negatives else None
        presort = {"on": side is not None}     # off for the per-kernel-event run (below)

        def loss_fn():
            neg = ops.draw_negatives(pos, cfg.num_posts, generator=gen)
            pre = None
            if presort["on"]:
                # the negatives' grouping by post needs only the edges and the draws: on a side
                # stream under the forward's gathers
                main = torch.cuda.current_stream(dev)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    pre = ops.presort_negatives(cfg.num_users, cfg.num_posts, pos, neg, "user")
                pre.rowptr.record_stream(main)
                pre.users.record_stream(main)
            out = model(g.x_dict, g.edge_index_dict)
            if presort["on"]:
                torch.cuda.current_stream(dev).wait_stream(side)
            return ops.edge_bce_loss(out["user"], out["post"], pos, neg, pw, neg_order="user",
                                     check=False, cscale=cscale, presorted=pre)
    else:
        env = parallel.DistEnv.from_torch()
        # every rank generates the seeded global graph's edges chunk by chunk on its own device
        # (counter-based draws: the same graph on every rank and at every N) and keeps only its
        # shard's (parallel.shard_edge_filter): the 200M-edge list never exists on one rank.
        # slice_inputs: every rank keeps the whole static input user table, so layer 1's post
        # slice mean is computed locally (no partial sums, no reduce-scatter at layer 1)
        keep = parallel.shard_edge_filter(cfg.num_users, cfg.num_posts, env.world, env.rank,
                                          slice_inputs=True)
        g = synth.make_graph(cfg, device=dev, device_gen=True, keep=keep)
        pos_g = g.edge_index_dict[synth.ENGAGES]
        pw_g = synth.interaction_weights(cfg.num_posts).to(dev)[pos_g[1]]
        n_eng = cfg.num_engages if cfg.num_engages else cfg.num_posts
        shard = parallel.UserShard({et: g.edge_index_dict[et] for et, _ in rels}, cfg.num_users,
                                   cfg.num_posts, env, impl=impl, pos_weights=pw_g,
                                   slice_inputs=True, num_edges_global=n_eng)
        x_user = g.x_dict["user"][shard.lo:shard.hi].contiguous()
        x_user_full = g.x_dict["user"]
        x_post = g.x_dict["post"]
        n_rel = {synth.ENGAGES: n_eng, synth.REV_ENGAGES: n_eng, synth.SOCIAL: cfg.num_social,
                 synth.POST_POST: cfg.num_post_post}
        edges_step = cfg.layers * sum(n_rel[et] for et, _ in rels)
        del g, pos_g, pw_g
        if not on_cpu:
            torch.cuda.empty_cache()
        model = HeteroSAGE(cfg.hidden, rels, num_layers=cfg.layers, in_channels=cfg.dim).to(dev)
        with torch.no_grad():
            shard.forward(model, x_user, x_post, x_user_full=x_user_full)
        for p in model.parameters():
            dist.broadcast(p.data, 0)

        def negatives():
            if on_cpu:
                return torch.randint(0, cfg.num_posts, (shard.pos_local.shape[1],),
                                     generator=gen, device=dev)
            return ops.draw_negatives(shard.pos_local, cfg.num_posts, generator=gen)

        def loss_fn():
            # the post table's last all-gather stays in flight under the negatives draw + sort
            h_u, h_p = shard.forward(model, x_user, x_post, wait=False, x_user_full=x_user_full)
            return shard.loss(h_u, h_p, negatives(), neg_order="user")

    # the reference's optimizer (train_gnn.py:207, Adam lr 0.001); on the GPU one native launch
    # over every parameter with --native-adam (optim.Adam), else torch's fused kernel
    opt = (optim.Adam(model.parameters(), lr=1e-3) if not on_cpu and args.native_adam
           else torch.optim.Adam(model.parameters(), lr=1e-3, fused=not on_cpu))

    def step():
        opt.zero_grad(set_to_none=True)
        if sharded and not args.autograd_sharded:
            # explicit schedule: each collective issued when its input is complete and waited
            # for by its consumer only (parallel.UserShard.step; same kernels and gradients)
            loss = shard.step(model, x_user, x_post, negatives(), neg_order="user",
                              x_user_full=x_user_full)
        else:
            loss = loss_fn()
            loss.backward()
        if sharded:
            parallel.sync_grads(model, parallel.DistEnv.from_torch())
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    clock = _Clock(dev, sharded, args, local)
    setup_s = time.perf_counter() - t_setup
    elapsed, loss = clock.time(step, args.steps)             # the headline: no events inside
    value = edges_step * args.steps / elapsed                 # edges_step is the global count
    # per-kernel HIP events: a separate run, so the headline carries none of their cost
    kern, timer_ms, dist_rec = {}, None, None
    if not args.profile_steps and args.timer_steps > 0 and (sharded or not on_cpu):
        # one stream: a kernel's events around its launch then time that kernel alone (the
        # negatives grouping, overlapped with the forward in the timed steps, runs in the loss).
        # N > 1: every collective's issue and its consumer's wait marked too (parallel.
        # CollectiveTrace), so the line says which collective stalled which rank
        if not sharded:
            presort["on"] = False
        timer = ops.KernelTimer() if not on_cpu else None
        trace = parallel.CollectiveTrace(dev) if sharded else None
        ops.set_timer(timer)
        parallel.set_collective_trace(trace)

        def traced_step():
            if trace is not None:
                trace.begin_step()
            return step()
        try:
            t_el, _ = clock.time(traced_step, args.timer_steps)
        finally:
            parallel.set_collective_trace(None)
            ops.set_timer(None)
        kern = timer.summary() if timer is not None else {}
        timer_ms = t_el / args.timer_steps * 1e3
        if trace is not None:
            dist_rec = _dist_summary(trace, kern, args.timer_steps, timer_ms, dev)
    # the reference's train() returns the global loss: sum the per-rank shares
    loss_t = loss.detach().to(torch.float64).reshape(1).clone()
    if sharded:
        dist.all_reduce(loss_t)
    if rank != 0:
        return None
    roof = _roofline(kern, cfg, world)
    if roof is not None and not on_cpu and not sharded:
        roof["one_pass"] = _one_pass_k1(g, cfg, roof)
    proj = _projection(kern, cfg.name)
    cpu = None
    if not args.no_cpu_baseline and world == 1 and not on_cpu and not sharded:
        if set(et for et, _ in rels) == {synth.ENGAGES, synth.REV_ENGAGES}:
            cpu = cpu_baseline_shard(cfg, g, rels, args.cpu_threads, args.cpu_shard,
                                     steps=args.cpu_steps)
        else:
            cpu = cpu_baseline(cfg, args.cpu_threads, args.cpu_sample_scale)
    strong = world == 1 or not args.weak
    return {
        "metric": "edges/s (fwd+bwd) hetero message-passing",
        "value": round(value, 1), "unit": "edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong" if strong else "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (seeded graph, uniform users / Zipf post degrees; random-init weights)",
        "config": {"workload": f"{cfg.name}: U={cfg.num_users} P={cfg.num_posts} "
                               f"E_engage={cfg.num_engages} (+reverse), "
                               f"relations={'+'.join(et[1] for et, _ in rels)}, "
                               f"d=h={cfg.dim}, "
                               f"{cfg.layers}-layer hetero-SAGE train step (fwd+loss+bwd+Adam)",
                   "edges_per_step": edges_step, "global_batch": edges_step,
                   "parallelism": (f"dst-partitioned x{world} (user shards + post-table slices: "
                                   "RCCL reduce-scatter / all-gather per layer)"
                                   if sharded else "single")},
        "roofline": roof, "projection": proj, "cpu_baseline": cpu, "dist": dist_rec,
        "kernel_timer": {"steps": args.timer_steps if kern else 0,
                         "ms_per_step": round(timer_ms, 3) if timer_ms else None,
                         "note": "per-kernel HIP events, separate run after the timed region, "
                                "every kernel on one stream (the timed steps group the loss's "
                                "negatives on a side stream under the forward)"},
        "kernels": _kernel_rows(kern, args.timer_steps, cfg.name, world),
        "kernels_note": ("GB/s = algorithmic bytes (SURVEY §8d) / HIP-event time; pmc_GB/s = "
                         "the committed PMC bytes (FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_r*.json) "
                         "/ the same time; cache_assisted: the algorithmic rate exceeds the 8 TB/s "
                         "peak, i.e. source rows come from L2 / the Infinity Cache"),
        "loss": float(loss_t),
        "setup_s": round(setup_s, 1),
    }


def _dist_summary(trace, kern, steps, step_ms, dev):
    """The N > 1 line's collective record (every rank calls this: it all-reduces): per collective
    position of the step, its op and buffer MB, the time from its issue to its consumer's wait
    completing (min / max over ranks), the stall it caused the consumer (min / max), the compute
    issued under it, and the buffer's delivery rate as the consumer saw it (a lower bound on the
    link rate: MB / the slowest rank's issue-to-wait time); per rank the compute ms per step (the
    per-kernel HIP events' sum; on the CPU rehearsal the step time minus the stalls) and the sum
    of its stalls.  The emulation's ``collectives`` / ``link_timeline`` measured for real."""
    rows = trace.per_position()
    M = torch.tensor([len(rows)], dtype=torch.int64, device=dev)
    m_min, m_max = M.clone(), M.clone()
    dist.all_reduce(m_min, op=dist.ReduceOp.MIN)
    dist.all_reduce(m_max, op=dist.ReduceOp.MAX)
    M = int(m_min)
    rows = rows[:M]
    v = torch.tensor([[r.get("wait_ms", 0.0), r.get("stall_ms", 0.0), r.get("cover_ms", 0.0)]
                      for r in rows] or [[0.0, 0.0, 0.0]], dtype=torch.float64, device=dev)
    stall_sum = sum(r.get("stall_ms", 0.0) for r in rows)
    compute = (sum(k["ms"] for k in kern.values()) / steps) if kern else step_ms - stall_sum
    per_rank = torch.tensor([[compute, stall_sum, step_ms]], dtype=torch.float64, device=dev)
    lo, hi = v.clone(), v.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    r_lo, r_hi = per_rank.clone(), per_rank.clone()
    dist.all_reduce(r_lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(r_hi, op=dist.ReduceOp.MAX)
    lo, hi, r_lo, r_hi = lo.tolist(), hi.tolist(), r_lo.tolist()[0], r_hi.tolist()[0]
    colls = []
    for j, r in enumerate(rows):
        mb = r["bytes"] / 1e6
        colls.append({"i": j, "op": r["op"], "MB": float(f"{mb:.4g}"),
                      "wait_ms_min": round(lo[j][0], 4), "wait_ms_max": round(hi[j][0], 4),
                      "stall_ms_min": round(lo[j][1], 4), "stall_ms_max": round(hi[j][1], 4),
                      "cover_ms_min": round(lo[j][2], 4),
                      "GBs": (float(f"{mb / 1e3 / (hi[j][0] * 1e-3):.4g}") if hi[j][0] > 0
                              else None)})
    return {"collectives_per_step": M, "positions_differ": bool(int(m_max) != M),
            "collectives": colls,
            "compute_ms_min": round(r_lo[0], 3), "compute_ms_max": round(r_hi[0], 3),
            "stall_ms_min": round(r_lo[1], 3), "stall_ms_max": round(r_hi[1], 3),
            "step_ms_min": round(r_lo[2], 3), "step_ms_max": round(r_hi[2], 3),
            "steps": steps,
            "compute_source": "per-kernel HIP events" if kern else "step time minus stalls",
            "note": ("per collective position of UserShard.step + the weight all-reduce, means over "
                     "the timer run's steps: wait = issue -> the consumer's wait done (cover + "
                     "stall), stall = the consumer stream's wait beyond its own work, cover = the "
                     "compute issued under it; GBs = the buffer MB / the slowest rank's wait (a "
                     "lower bound on the link rate); stall_ms = per rank, the sum over the step")}


def _pool_shapes(kern):
    """Mini-batch kernels change shape every batch: pool each kernel family over its launches
    (row counts replaced by '*'; bytes, flops and time summed)."""
    import re
    out = {}
    for k, v in kern.items():
        key = re.sub(r"(?<=\[)\d+|(?<=<-)\d+", "*", k)
        a = out.setdefault(key, {"launches": 0, "ms": 0.0, "bytes": 0, "cbytes": 0, "flops": 0})
        for f in a:
            a[f] += v[f]
    return out


def _roofline(kern, cfg, world, pooled=False):
    """The dominant HBM kernel: the K1 forward gather over the largest source table (the user
    table; at N>1 the weighted post partial sums over the rank's own users).  ``pooled``: the
    mini-batch kernels pooled over their shapes — the forward gather family with the most
    time."""
    fwd = {k: v for k, v in kern.items() if k.startswith(("gather_fwd", "gather_wfwd"))}
    if not fwd:
        return None
    if pooled:
        name = max(fwd, key=lambda k: fwd[k]["ms"])
    else:
        src_rows = lambda k: int(k.split("<-")[1].split("]")[0])
        name = max(fwd, key=lambda k: (src_rows(k), fwd[k]["ms"]))
    r = fwd[name]
    per_launch_ms = r["ms"] / r["launches"]
    per_launch_bytes = r["bytes"] / r["launches"]
    ach = per_launch_bytes / (per_launch_ms * 1e-3) / 1e9
    weighted = name.startswith("gather_wfwd")
    traffic, tsrc = _pmc_traffic(cfg.name, world, name)
    return {"bound": "hbm",
            "kernel": (f"k_gather K1 weighted fwd (post partial sums) {name}" if weighted
                       else f"k_gather K1 mean fwd {name}"),
            "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": tsrc, "avg_launch_us": round(per_launch_ms * 1e3, 1),
            "frac_note": ("frac = ALGORITHMIC bytes (SURVEY §8d: one source row per edge) per "
                          "launch over its time, cache-assisted: a launch is the source-block "
                          "passes (DESIGN §5) whose ~600 MB slices and the Zipf-hot rows reuse "
                          "L2 / the Infinity Cache, and PMC FETCH_SIZE counts Infinity-Cache "
                          "hits too; `traffic` is that PMC count (the passes' output round trips "
                          "included); `one_pass` is the unblocked gather"),
            "algorithmic_bytes_per_launch": int(per_launch_bytes),
            "bytes_formula": ("4*E*(2+d) + 4*(N_dst+1) + 4*N_dst*d" if weighted
                              else "4*E*(1+d) + 4*(N_dst+1) + 4*N_dst*d")}


def _one_pass_k1(g, cfg, roof):
    """The roofline kernel as ONE pass (no source blocking), timed with HIP events
    outside the timed region: the same algorithmic bytes over its own time."""
    from truth_recommendation_gnn_amd import graph as G, ops
    if not roof["kernel"].startswith("k_gather K1 mean fwd"):
        return None
    e = g.edge_index_dict[synth.ENGAGES]
    csr = G.relation_csr(e, cfg.num_users, cfg.num_posts)
    x = g.x_dict["user"]
    keep = ops.GATHER_BLOCK_BYTES
    ops.GATHER_BLOCK_BYTES = 0
    try:
        ops.gather_mean(x, csr)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(3):
            ops.gather_mean(x, csr)
        s1.record()
        torch.cuda.synchronize()
        ms = s0.elapsed_time(s1) / 3
    finally:
        ops.GATHER_BLOCK_BYTES = keep
    ach = roof["algorithmic_bytes_per_launch"] / (ms * 1e-3) / 1e9
    return {"avg_launch_us": round(ms * 1e3, 1), "achieved": round(ach, 1),
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "note": "the same gather in one pass over the 4.6 GB user table (HGNN_GATHER_BLOCK_GB=0)"}


MFMA_CLOCK_GHZ = 2.4         # MI355X_MICROARCH.md: peak engine clock the MFMA peaks are quoted at
N_SIMDS = 1024               # 256 CUs x 4 SIMDs
BF16_MFMA_CYCLES = 16        # v_mfma_f32_16x16x32_bf16 on one SIMD (16*16*32*2 flop / 1024 per cycle)


def _k3_roof(n, k, h, bytes_per_launch, x6):
    """The K3 launch's own floor in ms: max(its bytes over 8 TB/s, its matrix-core time).  On
    the bf16x6 split every 16x16x32 fp32 tile product is 6 ``v_mfma_f32_16x16x32_bf16`` of
    ``BF16_MFMA_CYCLES`` on one of the 1024 SIMDs at the peak clock; on the f32-input kernels
    the flops over the fp32 MFMA peak."""
    hbm_ms = bytes_per_launch / (HBM_PEAK_GBS * 1e9) * 1e3
    if x6:
        mfma = 6 * (n / 16) * (h / 16) * (k / 32)
        mfma_ms = mfma * BF16_MFMA_CYCLES / N_SIMDS / (MFMA_CLOCK_GHZ * 1e9) * 1e3
    else:
        mfma_ms = 2.0 * n * k * h / (FP32_MFMA_PEAK_TFS * 1e12) * 1e3
    return hbm_ms, mfma_ms


def _pmc_k3(cfg_name, n, k, fwd=True):
    """MFMA busy of the K3 launch from the newest committed K3 counter pass
    (profiles/pmc_k3_<cfg>_r<round>.json, scripts/pmc_k3_xs.sh: SQ_VALU_MFMA_BUSY_CYCLES over
    1024 SIMDs x the launch's GRBM_GUI_ACTIVE / 8), for the cfg4 step's 9M-row launches: the
    K = 256 forward has no added rows, the K = 128 forward is the pre-projected one (+ add)."""
    import glob
    base = cfg_name.split("x")[0]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"pmc_k3_{base}_r[0-9]*.json")),
                   key=lambda f: int(os.path.basename(f).rsplit("_r", 1)[1].split(".")[0]
                                     .split("_")[0]))
    files = [f for f in files if os.path.basename(f).rsplit("_r", 1)[1].split(".")[0].isdigit()]
    if not files or n != 9_000_000 or k not in (128, 256) or not fwd:
        return None, None
    key = f"k_lin_fwd_xs<{k}, {'true' if k == 128 else 'false'}>"
    with open(files[-1]) as f:
        rec = json.load(f).get("kernels", {}).get(key)
    if not rec or "mfma_util" not in rec:
        return None, None
    return rec["mfma_util"], f"profiles/{os.path.basename(files[-1])} {key}"


def _projection(kern, cfg_name=""):
    """The dense projection (K3), the largest forward launch, in fp32-GEMM-equivalent TFLOP/s
    (2*N*K*H per launch).  ``peak`` / ``frac``: against the chip's dense bf16 MFMA peak, which
    the fp32-exact bf16x6 split (6 bf16 products per fp32 product) turns into 2500 / 6 = 416.7
    fp32-equivalent TF/s, so ``frac`` = ``bf16_mfma_frac`` = 6 x achieved / 2500.  ``mfma_util``:
    the PMC matrix-pipe busy fraction of the same launch (committed K3 counter pass).
    ``frac_of_floor``: the launch's own floor — max(HBM bytes / 8 TB/s, its MFMA instructions'
    cycles at the peak clock), ``_k3_roof`` — over its time, with ``floor_rate`` the TF/s at
    that floor.  The f32-input kernels read against the fp32 MFMA peak instead."""
    lin = {k: v for k, v in kern.items() if k.startswith("linear_fwd[") and v["flops"]}
    if not lin:
        return None
    name = max(lin, key=lambda k: lin[k]["flops"] / lin[k]["launches"])
    r = lin[name]
    import re
    # "[NxK->H]", or "[*xK->H]" for the sampled blocks' varying row counts (cfg5)
    m = re.search(r"\[(\d+|\*)x(\d+)->(\d+)\]", name)
    k, h = (int(m.group(2)), int(m.group(3))) if m else (0, 0)
    x6 = (os.environ.get("HGNN_K3_X6", "1") != "0" and h == 128 and k in (128, 256, 384, 512))
    per_ms = r["ms"] / r["launches"]
    per_bytes = r["bytes"] / r["launches"]
    per_flops = r["flops"] / r["launches"]
    n = (int(m.group(1)) if m.group(1) != "*" else int(per_flops / (2 * k * h))) if m else 0
    hbm_ms, mfma_ms = _k3_roof(n, k, h, per_bytes, x6)
    floor_ms = max(hbm_ms, mfma_ms)
    tfs = per_flops / (per_ms * 1e-3) / 1e12
    peak = BF16_MFMA_PEAK_TFS / 6 if x6 else FP32_MFMA_PEAK_TFS
    util, util_src = _pmc_k3(cfg_name, n, k) if x6 else (None, None)
    out = {"bound": "hbm" if hbm_ms >= mfma_ms else "mfma", "kernel": f"k_linear_fwd K3 {name}",
           "achieved": round(tfs, 1), "peak": round(peak, 1),
           "unit": "TFLOP/s (fp32-GEMM equivalent)", "frac": round(tfs / peak, 4),
           "mfma_util": util, "mfma_util_source": util_src,
           "frac_of_floor": round(floor_ms / per_ms, 4),
           "floor_rate": round(per_flops / (floor_ms * 1e-3) / 1e12, 1),
           "floor_ms": {"hbm": round(hbm_ms, 4), "mfma": round(mfma_ms, 4)},
           "avg_launch_us": round(per_ms * 1e3, 1),
           "hbm_GB/s": round(per_bytes / (per_ms * 1e-3) / 1e9, 1),
           "flops_per_launch": int(per_flops),
           "flops_formula": "2*N*K*H (K = sum of the input segments)",
           "bytes_per_launch": int(per_bytes),
           "bytes_formula": "4*N*(K+H) (inputs read once, output written once; + 4*N*H for an added "
                            "row block, + 16*N for the ReLU mask bits)"}
    if x6:
        out["bf16_mfma_frac"] = round(6 * tfs / BF16_MFMA_PEAK_TFS, 4)
        out["method"] = ("bf16x6: fp32-exact 3-piece bf16 split, 6 v_mfma_f32_16x16x32_bf16 "
                         "products per fp32 product, f32 accumulate"
                         + (" (K > 256: two column-block launches, the second adding the "
                            "first's rows)" if k > 256 else ""))
        out["peak_note"] = (f"peak = the dense bf16 MFMA peak {BF16_MFMA_PEAK_TFS:g} TF/s / 6 "
                            "bf16 products per fp32 product; frac = bf16_mfma_frac = 6 x achieved "
                            "/ 2500")
        out["floor_note"] = (f"mfma floor = 6*(N/16)*(H/16)*(K/32) MFMAs x {BF16_MFMA_CYCLES} "
                             f"cycles / {N_SIMDS} SIMDs at {MFMA_CLOCK_GHZ} GHz (the launches "
                             "measured ~1.85 GHz under load, DESIGN §5); hbm floor = bytes / "
                             "8 TB/s")
    else:
        out["method"] = "f32-input MFMA (v_mfma_f32_16x16x4_f32)"
        out["peak_note"] = "peak = the dense fp32 MFMA peak"
    return out


def _kernel_rows(kern, steps, cfg_name, world):
    """The per-kernel table: algorithmic rate, compulsory rate, and where the committed PMC
    passes hold the kernel, the PMC byte rate beside them.  An algorithmic rate above the HBM
    peak is marked ``cache_assisted`` (its source rows hit L2 / the Infinity Cache)."""
    rows = {}
    for k, v in sorted(kern.items()):
        gbs = v["bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] else None
        ratio = _pmc_ratio(cfg_name, world, k)
        row = {"launches": v["launches"], "ms_per_step": round(v["ms"] / steps, 4),
               "GB/s": round(gbs, 1) if gbs is not None else None,
               "compulsory_GB/s": (round(v["cbytes"] / (v["ms"] * 1e-3) / 1e9, 1)
                                   if v["ms"] else None),
               "pmc_traffic_over_algorithmic": ratio,
               "pmc_GB/s": round(gbs * ratio, 1) if (gbs is not None and ratio) else None,
               "cache_assisted": bool(gbs is not None and gbs > HBM_PEAK_GBS)}
        if v["flops"] and v["ms"]:
            row["TFLOP/s"] = round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1)
        rows[k] = row
    return rows


# ----------------------------------------------------------------------------- cfg5 mini-batch
def _pad_rows(v, n):
    """The eager step's seed rows padded to the captured capacity (the link loss's shape)."""
    if int(v.shape[0]) == n:
        return v
    return torch.cat([v, v.new_zeros((n - int(v.shape[0]),) + tuple(v.shape[1:]))])


def _run_minibatch(args, dev, world, rank, local, sharded, impl):
    """BASELINE cfg5: the 4-relation graph (cfg4 + 90M user->user follows + 10M post->post),
    neighbour-sampled (fanout [15, 10], PyG NeighborLoader semantics, ``sampler.py``), one
    link-prediction mini-batch of ``--batch-seeds`` positive engages edges per rank per step
    (one uniform negative post each; seeds = their distinct endpoints): sample -> 2-layer hetero
    SAGE on the blocks (K1/K2/K3) -> the reference's link loss over the batch's pairs ->
    backward -> Adam.  N ranks are data-parallel (each holds the graph, takes its own slice of
    the epoch's edge order; one RCCL all-reduce of the weight gradients per step, between the
    two graph replays).  Edges = the sampled message edges of every block and relation (what the
    gathers aggregate), summed over ranks."""
    from truth_recommendation_gnn_amd import minibatch, ops, sampler
    if dev.type == "cpu":
        raise SystemExit("the cfg5 mini-batch bench runs the HIP sampler: no CPU rehearsal")
    cfg = synth.CONFIGS["cfg5"] if args.scale == 1.0 else synth.scaled("cfg5", args.scale)
    t_setup = time.perf_counter()
    g = synth.make_graph(cfg, device=dev, device_gen=True)
    rels = relations_of(cfg)
    fanouts = [15, 10]
    s = sampler.NeighborSampler({"user": cfg.num_users, "post": cfg.num_posts},
                                g.edge_index_dict, [et for et, _ in rels], fanouts)
    torch.manual_seed(synth.WEIGHT_SEED)
    model = HeteroSAGE(cfg.hidden, rels, num_layers=cfg.layers, in_channels=cfg.dim).to(dev)
    env = parallel.DistEnv.from_torch()
    if sharded:
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    # the step (forward, loss, backward, Adam) replayed as a HIP graph over static-capacity
    # blocks (minibatch.py); the sampler stays eager (two syncs per hop).  N > 1: the forward +
    # loss + backward graph, the eager all-reduce of the gradients, then the Adam graph.
    use_graph = not args.no_graph
    # the reference's Adam (train_gnn.py:207); --native-adam: one native launch over every
    # parameter, its step count on the device (optim.Adam: one graph node; torch's capturable
    # fused Adam: two)
    opt = (torch.optim.Adam(model.parameters(), lr=1e-3, fused=True, capturable=use_graph)
           if not args.native_adam or torch.device(dev).type != "cuda"
           else optim.Adam(model.parameters(), lr=1e-3))
    gen = torch.Generator(device=dev).manual_seed(0)
    gen_neg = torch.Generator(device=dev).manual_seed(1)
    # link prediction as a link loader does it: one shuffle of the positive (engages) edges per
    # epoch, each batch a slice of B of them; their endpoints and one uniform negative post per
    # positive (train_gnn.py:259-273) are the seeds
    pos_ei = g.edge_index_dict[synth.ENGAGES]
    n_pos = int(pos_ei.shape[1])
    order = torch.randperm(n_pos, device=dev, generator=gen, dtype=torch.int32)
    nb = args.batch_seeds
    per_epoch = n_pos // (nb * world)
    state = {"b": 0, "edges": 0}
    # the next batch is sampled on a side stream while this one's forward / backward runs: the
    # sampler's two host syncs per hop then wait for the sampling kernels only, not for the
    # previous step's GPU work queued ahead of them on one stream (a data loader's prefetch)
    # Eager, A/B on one box (round 3): 2.08 / 2.16 ms per step with it against 2.00 / 1.91
    # without — that step is bound by host issue, so it is off there.  Replaying the graph the
    # host is free during the step: 1.04 ms with it, 1.29-1.32 without — on by default.
    prefetch = args.prefetch or (use_graph and not args.no_prefetch)
    side = None
    if prefetch:
        side = _cu_masked_stream(dev, args.side_cus) if args.side_cus else torch.cuda.Stream(dev)
    if side is not None:
        # the setup above (the graph, the epoch's edge order) is queued on this stream: the side
        # stream must not read it before it is written (rounds 4-5 sampled the capture's batch
        # 0 from a half-written permutation)
        side.wait_stream(torch.cuda.current_stream(dev))

    ph = _Phases() if os.environ.get("HGNN_CFG5_PHASES") else None

    def sample(b, prep=True, eager=False):
        """Batch b on the side stream (when prefetching): staged by the sync-free LinkSampler
        (returns lb None), or — eager, before capture, ``--eager-sampler`` — a LinkBatch from
        link_batch + NeighborSampler.sample, staged by CapturedStep.prepare when ``prep``."""
        gb = (b % max(per_epoch, 1)) * world + rank            # this rank's slice of the order

        def make():
            # the edge ids made on the stream that samples them (rounds 4-5 cast them on the
            # main stream, behind the running replay, and the side stream read them unwritten)
            ids = order[gb * nb:(gb + 1) * nb].long()
            if ph:
                ph.mark(b, "smp0")
            if static is not None and not eager:
                with _Phases.host(ph, "sample"):
                    statics[b % len(statics)].prepare(ids, gb, gen_neg)
                if ph:
                    ph.mark(b, "smp1")
                    ph.mark(b, "prep1")
                return None
            with _Phases.host(ph, "link_batch"):
                lb = minibatch.link_batch(pos_ei, ids, cfg.num_posts, generator=gen_neg)
            with _Phases.host(ph, "sample"):
                lb.mb = s.sample(lb.seeds, seed=gb)
            if ph:
                ph.mark(b, "smp1")
            if prep:
                # the batch's block / loss structures into the staging buffers, on the same
                # stream as the sampler (the side stream under the running replay)
                with _Phases.host(ph, "prepare"):
                    if captured is not None:
                        captured.prepare(lb.mb, lb.pu, lb.pp, lb.pn)
                    else:
                        link_loss.prepare(lb.pu, lb.pp, lb.pn)
                if ph:
                    ph.mark(b, "prep1")
            return lb
        if side is None:
            return make(), None
        with torch.cuda.stream(side):
            lb = make()
        ev = torch.cuda.Event()
        ev.record(side)
        return lb, ev

    nxt = [None]
    # capacities: B user seeds, 2B post seeds (positives + negatives); a batch's distinct
    # endpoints fill a prefix, the rest are padded rows the loss never reads
    n_seeds = {"user": nb, "post": 2 * nb}
    link_loss = minibatch.LinkLoss(nb, n_seeds["user"], n_seeds["post"], dev, n_total=nb * world)

    def loss_for(ll):
        def loss_of(out):
            if args.torch_loss:
                u, p = out["user"], out["post"]
                pu, pp, pn = ll.uop.long(), ll.col.long(), ll.neg.long()
                pos = (u[pu] * p[pp]).sum(1)
                neg = (u[pu] * p[pn]).sum(1)
                return (torch.nn.functional.softplus(-pos).sum()
                        + torch.nn.functional.softplus(neg).sum()) / (nb * world)
            return ll(out)

        loss_of.make_csr = ll.make_csr           # fresh loss structures per recorded pass
        loss_of.prepare, loss_of.commit, loss_of.link_loss = ll.prepare, ll.commit, ll
        loss_of.use_padded_rows = ll.use_padded_rows   # the captured step's padded tables
        loss_of.partial_seeds = True             # both forms read the seed rows by local id
        return loss_of

    loss_of = loss_for(link_loss)

    # over RCCL the gradient all-reduce is recorded inside the step's graph (one replay per
    # step; with --dist at world 1 it is still issued, as a rehearsal of the captured
    # collective); gloo's collectives run on the host, so there it stays an eager call between
    # two replays
    capture_ar = (sharded and use_graph and args.dist_backend == "nccl" and dev.type == "cuda"
                  and not args.eager_allreduce)

    def sync():
        parallel.sync_grads(model, env, force=capture_ar)   # no-op at world size 1 otherwise

    captured = static = None
    caps, statics = [], []        # the captured step(s) and their LinkSamplers, used in turn
    edges_dev = torch.zeros((), dtype=torch.int64, device=dev)   # the LinkSampler's counts
    if use_graph:
        # the capture's two warm-up passes are training steps on batch 0 (then recorded once)
        captured = minibatch.CapturedStep(model, g.x_dict, s, n_seeds, loss_of, opt,
                                          between=sync if (world > 1 or capture_ar) else None,
                                          capture_between=capture_ar)
        lb0, ev0 = sample(0, prep=False)
        if ev0 is not None:
            # batch 0 came from the side stream: the capture's warm-up steps read it here
            # (rounds 4-5 did not wait, and their warm-up trained on a half-written batch 0)
            torch.cuda.current_stream(dev).wait_event(ev0)
            lb0.mb.record_stream(torch.cuda.current_stream(dev))
        link_loss.load(lb0.pu, lb0.pp, lb0.pn)
        captured.capture(lb0.mb, warmup=2)
        if _SERIAL:
            torch.cuda.synchronize()
            state["after_capture"] = [float(p.double().sum()) for p in model.parameters()][:4]
        caps = [captured]
        lls = [link_loss]
        if not args.eager_sampler and not args.single_buffer and captured.graph_opt is None:
            # a second recorded step over its own buffers: batches alternate between the two,
            # each sampled straight into the live buffers of the one not replaying — no staging
            # copy on the main stream (no warm-up: the first capture's steps are the training's)
            ll2 = minibatch.LinkLoss(nb, n_seeds["user"], n_seeds["post"], dev,
                                     n_total=nb * world)
            cap2 = minibatch.CapturedStep(model, g.x_dict, s, n_seeds, loss_for(ll2), opt,
                                          between=sync if (world > 1 or capture_ar) else None,
                                          capture_between=capture_ar)
            ll2.load(lb0.pu, lb0.pp, lb0.pn)
            cap2.capture(lb0.mb, warmup=0)
            caps.append(cap2)
            lls.append(ll2)
            for c, ll in zip(caps, lls):
                c.blocks.use_direct()
                ll.use_direct()
        if not args.eager_sampler:
            # every later batch: sampled straight into the staging buffers, no host sync
            statics = [minibatch.LinkSampler(c, pos_ei, cfg.num_posts, ll)
                       for c, ll in zip(caps, lls)]
            static = statics[0]
        torch.cuda.synchronize()   # setup done: its buffers are written before the side stream runs

    def eager(lb):
        link_loss.make_csr()
        out = sampler.forward_blocks(model, lb.mb, g.x_dict)
        loss = loss_of({t: v if t not in n_seeds else _pad_rows(v, link_loss.rows[t])
                        for t, v in out.items()})
        opt.zero_grad(set_to_none=True)
        loss.backward()
        sync()
        opt.step()
        return loss

    def step(graph=True):
        staged = graph and static is not None
        if nxt[0] is not None and (nxt[0][0] is None) != staged:
            nxt[0] = None                        # a prefetched batch of the other kind
        lb, ev = nxt[0] if nxt[0] is not None else sample(state["b"], eager=not staged)
        k = state["b"] % len(caps) if staged else 0
        state["b"] += 1
        main = torch.cuda.current_stream(dev)
        if ev is not None:
            main.wait_event(ev)
        if staged:
            edges_dev.add_(statics[k].edge_count())   # before the replay the next prepare waits on
        else:
            state["edges"] += sum(c.num_edges for blk in lb.mb.blocks for c in blk.csr.values())
        if _SERIAL and "stage0" not in state and captured is not None:
            torch.cuda.synchronize()
            state["stage0"] = [int(captured.blocks.arena._bytes["stage"].sum()),
                               int(link_loss.arena._bytes["stage"].sum())]
        if graph and captured is not None:
            if ph:
                ph.mark(state["b"] - 1, "rep0")
            with _Phases.host(ph, "step"):
                loss = caps[k].step()            # commit the staged batch (if staged), replay
            if ph:
                ph.mark(state["b"] - 1, "rep1")
        else:
            if ev is not None:                   # the eager step reads the batch on this stream
                lb.mb.record_stream(main)
                for t in (lb.pu, lb.pp, lb.pn):
                    t.record_stream(main)
            link_loss.commit()
            loss = eager(lb)
        if _SERIAL:
            torch.cuda.synchronize()
            state.setdefault("losses", []).append(float(loss))
        if side is not None:
            nxt[0] = sample(state["b"], eager=not staged)   # under this step's GPU work
            if _SERIAL:
                torch.cuda.synchronize()
        return loss

    # the steps (commit + replay) on a high-priority stream, the side stream's sampling at the
    # default (lowest) one: 0.852 / 0.850 vs 0.861 / 0.860 ms per batch (A/B, round 6)
    loop = (contextlib.nullcontext() if args.default_priority or dev.type != "cuda"
            else torch.cuda.stream(torch.cuda.Stream(dev, priority=-1)))
    with loop:
        for _ in range(args.warmup):
            step()
        setup_s = time.perf_counter() - t_setup
        clock = _Clock(dev, sharded, args, local)
        state["edges"] = 0
        edges_dev.zero_()
        if ph:
            ph.h.clear()
        elapsed, loss = clock.time(step, args.steps)
    edges = torch.tensor([float(state["edges"]) + float(edges_dev)], dtype=torch.float64,
                         device=dev)
    if sharded:
        dist.all_reduce(edges)
    edges = float(edges)
    phases = ph.summary(args.steps) if ph else None
    kern = {}
    if not args.profile_steps and args.timer_steps > 0:
        # per-kernel events need the eager launches: the timer steps run the same kernels
        # without the graph (on each batch's real sizes, not the static capacities)
        timer = ops.KernelTimer()
        ops.set_timer(timer)
        clock.time(lambda: step(graph=False), args.timer_steps)
        ops.set_timer(None)
        kern = timer.summary()
    if rank != 0:
        return None
    kern = _pool_shapes(kern)
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        lb, ev = nxt[0] if nxt[0] is not None else (None, None)
        if lb is None:                           # a LinkBatch of the next batch's edges
            lb, ev = sample(state["b"], prep=False, eager=True)
        if ev is not None:
            ev.synchronize()
        cpu = cpu_baseline_sampled(lb, g.x_dict, rels, cfg, args.cpu_threads)
    return {
        "metric": "edges/s (fwd+bwd) hetero message-passing",
        "value": round(edges / elapsed, 1), "unit": "edges/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (seeded graph; random-init weights)",
        "config": {"workload": f"{cfg.name} neighbour-sampled: U={cfg.num_users} "
                               f"P={cfg.num_posts} E_engage={cfg.num_engages} (+reverse) "
                               f"social={cfg.num_social} post_post={cfg.num_post_post}, "
                               f"d=h={cfg.dim}, fanout {fanouts}, link prediction: {nb} "
                               "positive engages edges + 1 uniform negative post each per rank "
                               "per step, seeds = their distinct endpoints; sample + 2-layer fwd "
                               "+ loss + bwd + Adam",
                   "edges_per_step": round(edges / args.steps),
                   "global_batch": nb * world,
                   "batches_per_s": round(world * args.steps / elapsed, 1),
                   "graph_replays_per_step": (None if captured is None else
                                              1 if captured.graph_opt is None else 2),
                   "graph_nodes": None if captured is None else captured.graph_nodes(),
                   "recorded_steps": len(caps) or None,
                   "parallelism": f"data-parallel x{world}" if world > 1 else "single",
                   "execution": ((("one HIP graph replay per step (forward + loss + backward + "
                                   "RCCL gradient all-reduce + Adam) over static-capacity blocks "
                                   if capture_ar else
                                   "one HIP graph replay per step over static-capacity blocks "
                                   if world == 1 else "HIP graph replays per step (forward + loss "
                                   "+ backward; eager gradient all-reduce; Adam) over "
                                   "static-capacity blocks")
                                  + ("" if static is not None else " (sampler eager)"))
                                 if captured is not None else "eager")
                   + (", next batch sampled on a side stream" if side is not None else "")
                   + (" by the sync-free LinkSampler straight into the staging buffers"
                      if static is not None else "")
                   + ("; two recorded steps replayed in turn, each batch sampled into the live "
                      "buffers of the one not replaying (no staging copy)" if len(caps) > 1
                      else "")},
        "roofline": _roofline(kern, cfg, world, pooled=True),
        "projection": _projection(kern, cfg.name),
        "cpu_baseline": cpu,
        "kernels": _kernel_rows(kern, args.timer_steps, cfg.name, world),
        "loss": float(loss.detach()), "setup_s": round(setup_s, 1),
        **({"phases": phases} if phases else {}),
        **({"losses": state.get("losses", [])[:40],
            "after_capture": state.get("after_capture"),
            "stage0": state.get("stage0")} if _SERIAL else {}),
    }


_SERIAL = os.environ.get("HGNN_CFG5_SERIAL") == "1"   # (diagnosis: no overlap of the streams)


def _cu_masked_stream(dev, n_cus: int):
    """A stream whose kernels run on the first ``n_cus`` compute units only
    (``hipExtStreamCreateWithCUMask``), wrapped for torch: the side stream's sampling then leaves
    the other CUs to the replay."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    n_total = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (n_total + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(min(n_cus, n_total)):
        mask[c // 32] |= 1 << (c % 32)
    stream = ctypes.c_void_p()
    with torch.cuda.device(dev):
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(stream), words, mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    return torch.cuda.ExternalStream(stream.value, device=dev)


class _Phases:
    """HGNN_CFG5_PHASES=1: where a cfg5 step's time goes — host seconds per phase of the loop
    (link batch, sampler, prepare, step issue) and, from events on the stream each phase runs
    on, the GPU spans per batch: sampling and prepare on the side stream, the replay on the
    main one, and the main stream's idle gap between two replays."""

    def __init__(self):
        self.h = {}
        self.ev = {}

    @staticmethod
    @contextlib.contextmanager
    def host(ph, name):
        if ph is None:
            yield
            return
        t = time.perf_counter()
        yield
        ph.h[name] = ph.h.get(name, 0.0) + time.perf_counter() - t

    def mark(self, b, name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.ev.setdefault(b, {})[name] = e

    def summary(self, steps):
        torch.cuda.synchronize()
        spans = {"sample": ("smp0", "smp1"), "prepare": ("smp1", "prep1"),
                 "replay": ("rep0", "rep1"), "prep_to_replay": ("prep1", "rep0")}
        out = {k: [] for k in list(spans) + ["main_idle"]}
        bs = sorted(b for b, e in self.ev.items() if {"smp0", "prep1", "rep0", "rep1"} <= set(e))
        for b in bs[-steps:]:
            e = self.ev[b]
            for k, (a, z) in spans.items():
                out[k].append(e[a].elapsed_time(e[z]))
            if b - 1 in self.ev and "rep1" in self.ev[b - 1]:
                out["main_idle"].append(self.ev[b - 1]["rep1"].elapsed_time(e["rep0"]))
        n = max(len(bs[-steps:]), 1)
        return {"host_ms_per_step": {k: round(v / n * 1e3, 4) for k, v in self.h.items()},
                "gpu_ms_mean": {k: round(sum(v) / max(len(v), 1), 4) for k, v in out.items()},
                "batches": n}


if __name__ == "__main__":
    main()
