"""Experiment: K1 over the cfg4 post <- user relation (200M edges, 9M x 128 fp32 source table =
4.6 GB) as one pass vs B passes, pass b summing only the sources of user block b (a 4.6/B GB
slice: at B >= 24 it fits the 256 MB Infinity Cache), accumulating into the output.  Prints
ms per full gather for each B.  usage: python scripts/ic_block_bench.py [B ...]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from truth_recommendation_gnn_amd import graph, ops, synth  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    dev = torch.device("cuda")
    cfg = synth.CONFIGS["cfg4"]
    t0 = time.time()
    g = synth.make_graph(cfg, device=dev, device_gen=True)
    ei = g.edge_index_dict[synth.ENGAGES]            # user -> post
    n_u, n_p = cfg.num_users, cfg.num_posts
    x = g.x_dict["user"]
    del g
    print(f"graph {time.time() - t0:.1f}s E={ei.shape[1]}", flush=True)
    csr = graph.relation_csr(ei, n_u, n_p)
    ref = torch.empty(n_p, x.shape[1], device=dev)
    t_one = timed(lambda: ops._gather(x, csr.fwd, None, False, ref, False))
    print(f"B=1 {t_one:.3f} ms  heavy={csr.fwd.plan.n_heavy}", flush=True)
    Bs = [int(b) for b in sys.argv[1:]] or [8, 16, 24, 32, 48]
    for B in Bs:
        bs = -(-n_u // B)
        key = (ei[0] // bs) * n_p + ei[1]
        ge = graph.group_edges(key, ei[0], B * n_p, n_u)
        del key
        parts = []
        for b in range(B):
            rp = ge.rowptr[b * n_p:(b + 1) * n_p + 1]
            parts.append(graph.GroupedEdges(rp, ge.col, ge.perm,
                                            graph._plan(rp, n_p, ge.plan.chunk), n_p))
        out = torch.empty_like(ref)

        def run():
            for b, gb in enumerate(parts):
                ops._gather(x, gb, None, False, out, b > 0)
        t = timed(run)
        err = float((out - ref).abs().max() / ref.abs().max())
        print(f"B={B} {t:.3f} ms ({t_one / t:.2f}x)  rel_err={err:.2e}  "
              f"heavy={sum(p.plan.n_heavy for p in parts)}", flush=True)
        del ge, parts, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
