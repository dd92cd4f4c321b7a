"""Experiment: the random-row rate of the cfg4 post <- user gather (200M edges over 9M user rows)
as a function of the row width: one K1 pass over a 9M x d fp32 table for d = 64, 128, 256.  If
1-KiB rows stream faster than 512-B rows, two user-side tables read by gathers over the same
edges (the loss's dP gather reads U, the K2 into the posts reads dz) would gain from one
interleaved [U | dz] table.  usage: python scripts/row_width_bench.py"""
import sys
import time

import torch

sys.path.insert(0, ".")
from truth_recommendation_gnn_amd import graph, ops, synth  # noqa: E402
from scripts.ic_block_bench import timed  # noqa: E402


def main():
    dev = torch.device("cuda")
    cfg = synth.CONFIGS["cfg4"]
    t0 = time.time()
    g = synth.make_graph(cfg, device=dev, device_gen=True)
    ei = g.edge_index_dict[synth.ENGAGES]
    del g
    csr = graph.relation_csr(ei, cfg.num_users, cfg.num_posts)
    E = int(ei.shape[1])
    print(f"graph {time.time() - t0:.1f}s E={E}", flush=True)
    for d in (64, 128, 256):
        x = torch.randn(cfg.num_users, d, device=dev)
        out = torch.empty(cfg.num_posts, d, device=dev)
        ms = timed(lambda: ops._gather(x, csr.fwd, None, False, out, False))
        gb = (E * (4 * d + 4) + cfg.num_posts * 4 * d) / 1e9
        print(f'{{"d": {d}, "ms": {ms:.3f}, "GB": {gb:.1f}, "GB/s": {gb / ms * 1e3:.0f}}}',
              flush=True)
        del x, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
