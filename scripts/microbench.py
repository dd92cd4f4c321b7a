#!/usr/bin/env python3
"""Per-kernel timing of the cfg2 step on one GPU (HIP events on the launch stream), so each
kernel can be priced against its own roofline.  python scripts/microbench.py [--config cfg2]"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import graph, ops, synth  # noqa: E402
from truth_recommendation_gnn_amd import _native as N  # noqa: E402


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda")
    cfg = synth.CONFIGS[args.config]
    g = synth.make_graph(cfg, device=dev)
    U, P = g.x_dict["user"], g.x_dict["post"]
    d = cfg.dim
    eng = g.edge_index_dict[synth.ENGAGES]
    rev = g.edge_index_dict[synth.REV_ENGAGES]
    c_eng = graph.relation_csr(eng, cfg.num_users, cfg.num_posts)
    c_rev = graph.relation_csr(rev, cfg.num_posts, cfg.num_users)
    _ = c_eng.bwd, c_rev.bwd
    E = c_eng.num_edges
    res = {}

    def rec(name, ms, nbytes=None):
        r = {"ms": round(ms, 4)}
        if nbytes:
            r["GB/s"] = round(nbytes / (ms * 1e-3) / 1e9, 1)
        res[name] = r
        print(f"{name:40s} {ms * 1e3:9.1f} us" + (f"  {r['GB/s']:8.1f} GB/s" if nbytes else ""),
              flush=True)

    for nm, csr, x in (("K1 fwd rev (dst=user, src=post)", c_rev, P),
                       ("K1 fwd eng (dst=post, src=user)", c_eng, U)):
        rec(nm, timeit(lambda: ops.gather_mean(x, csr), args.reps),
            ops.gather_bytes(E, csr.n_dst, d, False))
        print("   heavy rows:", csr.fwd.plan.n_heavy, "chunks:", csr.fwd.plan.n_chunks,
              "chunk:", csr.fwd.plan.chunk)
    gU = torch.randn_like(U)
    gP = torch.randn_like(P)
    rec("K2 bwd rev (grad->post via CSC)", timeit(lambda: ops.scatter_mean_bwd(gU, c_rev), args.reps),
        ops.gather_bytes(E, cfg.num_posts, d, True))
    rec("K2 bwd eng (grad->user via CSC)", timeit(lambda: ops.scatter_mean_bwd(gP, c_eng), args.reps),
        ops.gather_bytes(E, cfg.num_users, d, True))

    # linear
    A_u, A_p = torch.randn_like(U), torch.randn_like(P)
    W = torch.randn(cfg.hidden, 2 * d, device=dev) * 0.1
    b = torch.randn(cfg.hidden, device=dev)
    rec("K3 fwd user (2 seg)", timeit(lambda: ops.linear_fwd([A_u, U], W, b, True), args.reps),
        4 * cfg.num_users * (2 * d + cfg.hidden))
    rec("K3 fwd post (2 seg)", timeit(lambda: ops.linear_fwd([A_p, P], W, b, True), args.reps),
        4 * cfg.num_posts * (2 * d + cfg.hidden))
    out_u = ops.linear_fwd([A_u, U], W, b, True)
    dout = torch.randn_like(out_u)
    dA, dX = torch.empty_like(A_u), torch.empty_like(U)
    rec("K3 bwd user dgrad+wgrad", timeit(lambda: ops.linear_bwd([A_u, U], W, dout, out_u,
                                                                 [dA, dX], True, True), args.reps),
        4 * cfg.num_users * (2 * cfg.hidden + 4 * d))
    rec("K3 bwd user wgrad only", timeit(lambda: ops.linear_bwd([A_u, U], W, dout, out_u,
                                                                [None, None], True, True), args.reps),
        4 * cfg.num_users * (2 * cfg.hidden + 2 * d))
    rec("K3 bwd user dgrad only", timeit(lambda: ops.linear_bwd([A_u, U], W, dout, out_u,
                                                                [dA, dX], False, False), args.reps),
        4 * cfg.num_users * (2 * cfg.hidden + 2 * d))

    # loss
    pw = synth.interaction_weights(cfg.num_posts).to(dev)[eng[1]]
    gen = torch.Generator(device=dev).manual_seed(3)
    neg = ops.sample_negatives(eng, cfg.num_posts, generator=gen)
    Ug, Pg = U.clone().requires_grad_(), P.clone().requires_grad_()

    def loss_fwd():
        return ops.edge_bce_loss(Ug, Pg, eng, neg, pw, neg_order="user", check=False)
    rec("loss fwd total (A+sort+2 gathers)", timeit(loss_fwd, args.reps))
    t = ops.KernelTimer()
    ops.set_timer(t)
    for _ in range(args.reps):
        loss_fwd()
    ops.set_timer(None)
    for k, v in t.summary().items():
        rec("  loss/" + k, v["ms"] / v["launches"] * (v["launches"] / args.reps),
            v["bytes"] / args.reps)
    # evaluation (train_gnn.py:289-367): 10% of the engages as test edges
    from truth_recommendation_gnn_amd import metrics
    te = eng[:, ::10].clone()
    te[1] += cfg.num_users
    n_eval_users = int(torch.unique(te[0]).numel())
    ms = timeit(lambda: metrics.evaluate(te, U, P, K=10), 2, 1)
    rec("evaluate Recall/NDCG@10 (10% test)", ms)
    print(f"   test users {n_eval_users}, candidates {int(torch.unique(te[1]).numel())}")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
