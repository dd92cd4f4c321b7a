#!/usr/bin/env python3
"""f3 evaluation at cfg2 scale (train_gnn.py:289-367): 10% of the engages as test edges, the
cfg2 feature tables as embeddings (d=64; --dim 128 pads them to d=128 with fresh columns).

Times ``metrics.evaluate`` on the fused path (hgnn_score_topk + hgnn_topk_finish) and on the
materialised path (hipBLASLt GEMM per user batch + hgnn_topk_metrics), checks they agree, and
prices the fused kernel against the fp32 MFMA peak (2·rows·C·d flop per launch).
python scripts/eval_bench.py [--dim 64|128]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import _native as N, metrics, synth  # noqa: E402

MFMA_F32_PEAK_TFLOPS = 157.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda")
    cfg = synth.CONFIGS["cfg2"]
    g = synth.make_graph(cfg, device=dev)
    U, P = g.x_dict["user"], g.x_dict["post"]
    if args.dim != U.shape[1]:
        gen = torch.Generator(device=dev).manual_seed(7)
        extra = args.dim - U.shape[1]
        U = torch.cat([U, torch.randn(U.shape[0], extra, device=dev, generator=gen) * 0.1], 1)
        P = torch.cat([P, torch.randn(P.shape[0], extra, device=dev, generator=gen) * 0.1], 1)
    te = g.edge_index_dict[synth.ENGAGES][:, ::10].clone()
    te[1] += cfg.num_users
    res = {"dim": args.dim}
    for fused in (True, False):
        out = metrics.evaluate(te, U, P, K=10, fused=fused)   # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            out = metrics.evaluate(te, U, P, K=10, fused=fused)
        torch.cuda.synchronize()
        res["fused" if fused else "materialised"] = {
            "ms": round((time.perf_counter() - t0) / args.reps * 1e3, 2),
            "recall@10": out[0], "ndcg@10": out[1]}
    # the fused kernel alone, HIP events on the launch stream
    grp = metrics._Grouped(te, cfg.num_users, cfg.num_posts)
    n_rows, C = int(grp.users.numel()), int(grp.cand.numel())
    Pc = P.index_select(0, grp.cand).contiguous()
    users32 = grp.users.to(torch.int32)
    topv = torch.empty(n_rows, 11, device=dev)
    topi = torch.empty(n_rows, 11, dtype=torch.int32, device=dev)
    lib = N.lib()
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ms = []
    for _ in range(args.reps + 1):
        ev[0].record(st)
        N.check(lib.hgnn_score_topk(N.ptr(U), N.ptr(users32), n_rows, N.ptr(Pc), C, args.dim, 11,
                                    N.ptr(topv), N.ptr(topi), N.stream_ptr(dev)), "score_topk")
        ev[1].record(st)
        torch.cuda.synchronize()
        ms.append(ev[0].elapsed_time(ev[1]))
    k_ms = sorted(ms[1:])[len(ms[1:]) // 2]
    flop = 2.0 * n_rows * C * args.dim
    res["rows"], res["candidates"] = n_rows, C
    res["score_topk_kernel"] = {"ms": round(k_ms, 3), "TFLOP/s": round(flop / k_ms / 1e9, 1),
                                "mfma_frac": round(flop / k_ms / 1e9 / MFMA_F32_PEAK_TFLOPS, 3)}
    f, m = res["fused"], res["materialised"]
    res["agree"] = abs(f["recall@10"] - m["recall@10"]) < 1e-4 and \
        abs(f["ndcg@10"] - m["ndcg@10"]) < 1e-4
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
