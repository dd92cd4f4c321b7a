#!/usr/bin/env python3
"""Negatives-sort microbench (HIP events): ``--mode sort`` = hgnn_uniform_i32 + hgnn_sort_pairs_i32
(two calls), ``--mode draw`` = hgnn_draw_sort_negatives (draws inside the first pass), on E
uniform keys in [0, n_keys) with the user-of-position payload (the loss's (post, user) grouping;
defaults: cfg4, 200M negatives over 1M posts)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--edges", type=int, default=200_000_000)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--mode", choices=["sort", "draw", "both"], default="both")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    seed = torch.tensor([12345], dtype=torch.int64, device=dev)
    # user of position: sorted user ids, ~22 positions per user as at cfg4
    pay = torch.sort(torch.randint(0, max(1, a.edges // 22), (a.edges,), device=dev,
                                   dtype=torch.int32))[0]
    neg = torch.empty(a.edges, dtype=torch.int32, device=dev)
    rowptr = torch.empty(a.keys + 1, dtype=torch.int32, device=dev)
    out = torch.empty(a.edges, dtype=torch.int32, device=dev)
    lib = N.lib()
    ws = N.workspace(lib.hgnn_sort_pairs_ws_bytes(a.edges, a.keys), dev)
    s = N.stream_ptr(dev)

    def run_sort():
        N.check(lib.hgnn_uniform_i32(N.ptr(seed), a.edges, a.keys, N.ptr(neg), s), "uniform")
        N.check(lib.hgnn_sort_pairs_i32(N.ptr(neg), N.ptr(pay), None, a.edges, a.keys,
                                        N.ptr(rowptr), N.ptr(out), None, None, N.ptr(ws),
                                        ws.numel(), s), "sort")

    def run_draw():
        N.check(lib.hgnn_draw_sort_negatives(N.ptr(seed), N.ptr(pay), a.edges, a.keys, N.ptr(neg),
                                             N.ptr(rowptr), N.ptr(out), N.ptr(ws), ws.numel(), s),
                "draw_sort")

    modes = ["sort", "draw"] if a.mode == "both" else [a.mode]
    res = {}
    for m in modes:
        fn = run_sort if m == "sort" else run_draw
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        res[m] = (out.clone(), rowptr.clone())
        print(f"{m}: E={a.edges} keys={a.keys} {ms * 1e3:.1f} us  "
              f"{a.edges / ms / 1e6:.2f} Gkeys/s", flush=True)
    if len(res) == 2:
        print("identical:", all(torch.equal(x, y) for x, y in zip(res["sort"], res["draw"])))


if __name__ == "__main__":
    main()
