#!/usr/bin/env python3
"""K3 forward/backward A/B at one cfg4 shape (HIP events): the kernel version comes from the
environment (HGNN_K3_FWD=4..11, HGNN_K3_DGRAD, HGNN_K3_WGRAD: read once per process), so run one
process per version.  python scripts/k3_ab.py --rows 9000000 --k 128 --h 128 [--add] [--bwd]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import ops  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=9_000_000)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--h", type=int, default=128)
    ap.add_argument("--segs", type=int, default=1, help="input split into this many segments")
    ap.add_argument("--add", action="store_true")
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--no-mask", action="store_true", help="no ReLU bit mask output")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    n, k, h = a.rows, a.k, a.h
    segs = [torch.randn(n, k // a.segs, device=dev, generator=g) for _ in range(a.segs)]
    w = torch.randn(h, k, device=dev, generator=g) * 0.1
    b = torch.randn(h, device=dev, generator=g)
    add = torch.randn(n, h, device=dev, generator=g) if a.add else None
    mk = None if a.no_mask else ops.relu_mask_for(n, h, True, dev)
    out = ops.linear_fwd(segs, w, b, True, add=add, mask_out=mk)
    ref = torch.addmm(b, torch.cat(segs, 1), w.t())
    if add is not None:
        ref += add
    ref.relu_()
    err = float((out - ref).abs().max() / ref.abs().max())
    del ref
    ms = timeit(lambda: ops.linear_fwd(segs, w, b, True, add=add, mask_out=mk), a.reps)
    fl = 2 * n * k * h
    rec = {"shape": f"{n}x{k}->{h}" + ("+add" if a.add else ""),
           "fwd_ver": os.environ.get("HGNN_K3_FWD", "default"), "fwd_ms": round(ms, 3),
           "fwd_TFs": round(fl / ms / 1e9, 1), "fwd_frac_of_155": round(fl / ms / 1e9 / 155.1, 3),
           "max_rel_err_vs_torch": float(f"{err:.2e}")}
    if a.bwd:
        dout = torch.randn(n, h, device=dev, generator=g)
        dxs = [torch.empty_like(s) for s in segs]
        ms_b = timeit(lambda: ops.linear_bwd(segs, w, dout, out, dxs, True, True, mask=mk), a.reps)
        rec.update({"bwd_ms": round(ms_b, 3), "bwd_TFs": round(2 * fl / ms_b / 1e9, 1),
                    "bwd_frac_of_155": round(2 * fl / ms_b / 1e9 / 155.1, 3),
                    "dgrad_ver": os.environ.get("HGNN_K3_DGRAD", "default"),
                    "wgrad_ver": os.environ.get("HGNN_K3_WGRAD", "default")})
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
