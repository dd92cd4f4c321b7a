"""A/B of the loss's dP gather at cfg4: one pass over the 4.6 GB user table
(hgnn_score_gather2, nt row loads) against B source-block passes (ops._score_gather2_blocked:
the positives from the K1 blocks of the same relation, the negatives split per block by
hgnn_segment_bounds, passes 2.. accumulating; default-policy or nt row loads).  Times the
`score_gather` entry of ops.KernelTimer inside the real loss call (same launches the bench
step issues) and checks each variant's dP against the one pass.  One JSON line per variant.
usage: python scripts/score_block_bench.py [B:cached ...]   (default 1:1 8:1 8:0 4:1 12:1)"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from truth_recommendation_gnn_amd import ops, synth  # noqa: E402


def main():
    dev = torch.device("cuda")
    cfg = synth.CONFIGS["cfg4"]
    t0 = time.time()
    g = synth.make_graph(cfg, device=dev, device_gen=True)
    pos = g.edge_index_dict[synth.ENGAGES]
    n_u, n_p, d = cfg.num_users, cfg.num_posts, cfg.hidden
    del g
    gen = torch.Generator(device=dev).manual_seed(3)
    U = torch.randn(n_u, d, device=dev, generator=gen) * 0.1
    P = torch.randn(n_p, d, device=dev, generator=gen) * 0.1
    neg = ops.draw_negatives(pos, n_p, generator=gen)
    c = torch.tensor(1.3, device=dev)
    E = int(pos.shape[1])
    print(f"setup {time.time() - t0:.1f}s", flush=True)
    variants = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:]] or \
        [(1, 1), (8, 1), (8, 0), (4, 1), (12, 1)]
    ref = None
    for B, cached in variants:
        ops.DP_BLOCKS, ops.DP_CACHED = str(B), bool(cached)
        out = ops.edge_bce_loss_raw(U, P, pos, neg, E, c)        # warm-up (blocks built here)
        dp = out[2].clone()
        del out
        timer = ops.KernelTimer()
        ops.set_timer(timer)
        reps = 3
        for _ in range(reps):
            out = ops.edge_bce_loss_raw(U, P, pos, neg, E, c)
            del out
        ops.set_timer(None)
        summ = timer.summary()
        k = [n for n in summ if n.startswith("score_gather")][0]
        ms = summ[k]["ms"] / summ[k]["launches"]
        gbs = summ[k]["bytes"] / summ[k]["launches"] / (ms * 1e-3) / 1e9
        rec = {"B": B, "cached_loads": bool(cached) if B > 1 else False, "dp_gather_ms": round(ms, 3),
               "algorithmic_GB/s": round(gbs, 1), "frac_8TBs": round(gbs / 8000, 4),
               "edge_score_ms": round(summ["edge_score_d128"]["ms"] / reps, 3)}
        if ref is None and B == 1:
            ref = dp
        if ref is not None:
            rec["dP_rel_err_vs_one_pass"] = float((dp - ref).abs().max() / ref.abs().max())
        print(json.dumps(rec), flush=True)
        del dp
    ops.DP_BLOCKS = "1"


if __name__ == "__main__":
    main()
