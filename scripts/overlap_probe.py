#!/usr/bin/env python3
"""Probe: can the cache-bound user<-post K1 gather and the K3 user projection share the chip?
Times each alone and both launched together on two streams (independent inputs, cfg2 shapes).
If together ~ max(alone), a fused gather+projection kernel has room; if ~ sum, it does not."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import graph, ops, synth  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = torch.device("cuda")
    cfg = synth.CONFIGS["cfg2"]
    g = synth.make_graph(cfg, device=dev)
    P = g.x_dict["post"]
    rev = g.edge_index_dict[synth.REV_ENGAGES]
    c_rev = graph.relation_csr(rev, cfg.num_posts, cfg.num_users)
    n, d, h = cfg.num_users, 64, 64
    A = torch.randn(n, d, device=dev)
    X = torch.randn(n, d, device=dev)
    W = torch.randn(h, 2 * d, device=dev) * 0.1
    b = torch.randn(h, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    k1 = lambda: ops.gather_mean(P, c_rev)
    k3 = lambda: ops.linear_fwd([A, X], W, b, True)

    def both():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            k1()
        with torch.cuda.stream(s2):
            k3()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    t1, t3, tb = timeit(k1), timeit(k3), timeit(both)
    print(f"K1 user<-post alone {t1:.1f} us, K3 alone {t3:.1f} us, sum {t1 + t3:.1f}, "
          f"together {tb:.1f} us", flush=True)


if __name__ == "__main__":
    main()
