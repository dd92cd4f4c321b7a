"""Experiment: K1 over the cfg4 post <- user relation (200M edges, 9M x 128 fp32 source table =
4.6 GB) as one pass vs B x D passes: pass (d, b) sums, for the destination rows of group d (D
contiguous ranges of posts), only the sources in user block b (a 4.6/B GB slice), accumulating
into the output.  D > 1 keeps each group's accumulator (512/D MB) cache-resident across its B
passes.  IC_REV=1: the user <- post relation (the 512 MB post table) instead.  Prints ms per
full gather.  usage: [IC_REV=1] python scripts/ic_block_bench.py [B:D ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from truth_recommendation_gnn_amd import graph, ops, synth  # noqa: E402


def timed(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda")
    cfg = synth.CONFIGS["cfg4"]
    t0 = time.time()
    g = synth.make_graph(cfg, device=dev, device_gen=True)
    rev = os.environ.get("IC_REV", "0") == "1"       # the user <- post relation instead
    ei = g.edge_index_dict[synth.REV_ENGAGES if rev else synth.ENGAGES]
    n_u, n_p = cfg.num_users, cfg.num_posts
    x = g.x_dict["post" if rev else "user"]
    if rev:                                           # sources: posts, destinations: users
        n_u, n_p = n_p, n_u
    del g
    print(f"graph {time.time() - t0:.1f}s E={ei.shape[1]}", flush=True)
    csr = graph.relation_csr(ei, n_u, n_p)
    ref = torch.empty(n_p, x.shape[1], device=dev)
    t_one = timed(lambda: ops._gather(x, csr.fwd, None, False, ref, False))
    print(f"B=1 D=1 {t_one:.3f} ms", flush=True)
    specs = sys.argv[1:] or ["8:1", "16:1", "8:2", "8:4", "16:4", "16:8", "24:8", "32:8"]
    for spec in specs:
        B, D = (int(v) for v in spec.split(":"))
        bs = -(-n_u // B)
        key = (ei[0] // bs) * n_p + ei[1]
        ge = graph.group_edges(key, ei[0], B * n_p, n_u)
        del key
        ds = -(-n_p // D)
        parts = []
        for d in range(D):
            lo, hi = d * ds, min((d + 1) * ds, n_p)
            for b in range(B):
                rp = ge.rowptr[b * n_p + lo:b * n_p + hi + 1]
                parts.append((lo, hi, b, graph.GroupedEdges(
                    rp, ge.col, ge.perm, graph._plan(rp, hi - lo, ge.plan.chunk), hi - lo)))
        out = torch.empty_like(ref)

        def run():
            for lo, hi, b, gb in parts:
                ops._gather(x, gb, None, False, out[lo:hi], b > 0)
        t = timed(run)
        err = float((out - ref).abs().max() / ref.abs().max())
        print(f"B={B} D={D} {t:.3f} ms ({t_one / t:.3f}x)  rel_err={err:.2e}", flush=True)
        del ge, parts, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
