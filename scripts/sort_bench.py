#!/usr/bin/env python3
"""Negatives-sort microbench: hgnn_sort_pairs_i32 on E uniform int32 keys in [0, n_keys) with one
payload (the loss's (post, user) sort at cfg2), HIP-event timed.  HGNN_SORT_LSD=1 selects the
counting-pass LSD sort instead of onesweep (read once per process)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--keys", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    k = torch.randint(0, a.keys, (a.edges,), device=dev, generator=g, dtype=torch.int32)
    pay = torch.randint(0, 1 << 20, (a.edges,), device=dev, generator=g, dtype=torch.int32)
    rowptr = torch.empty(a.keys + 1, dtype=torch.int32, device=dev)
    out = torch.empty(a.edges, dtype=torch.int32, device=dev)
    lib = N.lib()
    ws = N.workspace(lib.hgnn_sort_pairs_ws_bytes(a.edges, a.keys), dev)
    s = N.stream_ptr(dev)

    def run():
        N.check(lib.hgnn_sort_pairs_i32(N.ptr(k), N.ptr(pay), None, a.edges, a.keys, N.ptr(rowptr),
                                        N.ptr(out), None, None, N.ptr(ws), ws.numel(), s), "sort")
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    ref = torch.sort(k.long() * (1 << 31) + torch.arange(a.edges, device=dev))[1]
    ok = torch.equal(out, pay[ref])
    mode = "lsd" if os.environ.get("HGNN_SORT_LSD") == "1" else "onesweep"
    print(f"{mode}: E={a.edges} keys={a.keys} {ms * 1e3:.1f} us/sort  "
          f"{a.edges / ms / 1e6:.2f} Gkeys/s  correct={ok}", flush=True)


if __name__ == "__main__":
    main()
