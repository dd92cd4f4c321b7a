#!/usr/bin/env python3
"""K3 microbench: the fused multi-segment linear at the cfg2 / cfg3 user-side shapes (N = 1M
rows, two segments [aggregate | root]), forward and backward (fused dgrad+wgrad; wgrad only),
HIP-event timed; TFLOP/s against the 157 TF/s fp32 MFMA peak and HBM GB/s.
python scripts/k3_bench.py [--rows 1000000] [--reps 20]"""
import argparse
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
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dims", default="64,128", help="d = h values to time")
    ap.add_argument("--shapes", default=None,
                    help="K:H pairs, e.g. 128:128,256:128 (K = two segments of K/2); "
                         "overrides --dims")
    ap.add_argument("--check", action="store_true", help="check outputs against float64 torch")
    a = ap.parse_args()
    dev = torch.device("cuda")
    n = a.rows
    shapes = ([tuple(int(v) for v in x.split(":")) for x in a.shapes.split(",")] if a.shapes
              else [(2 * int(x), int(x)) for x in a.dims.split(",")])
    for kk, h in shapes:
        d = kk // 2
        g = torch.Generator(device=dev).manual_seed(0)
        A = torch.randn(n, d, device=dev, generator=g)
        X = torch.randn(n, d, device=dev, generator=g)
        W = torch.randn(h, 2 * d, device=dev, generator=g) * 0.1
        b = torch.randn(h, device=dev, generator=g)
        out = ops.linear_fwd([A, X], W, b, True)
        ref = torch.relu(torch.cat([A, X], 1) @ W.T + b)
        err = float((out - ref).abs().max() / ref.abs().max())
        dout = torch.randn_like(out)
        dA, dX = torch.empty_like(A), torch.empty_like(X)
        k = 2 * d
        fl = 2 * n * k * h
        t = timeit(lambda: ops.linear_fwd([A, X], W, b, True), a.reps)
        print(f"fwd  K={k} H={h}: {t * 1e3:7.1f} us  {fl / t / 1e9:6.1f} TF/s  "
              f"{4 * n * (k + h) / t / 1e6:6.0f} GB/s  (rel err {err:.1e})", flush=True)
        t = timeit(lambda: ops.linear_bwd([A, X], W, dout, out, [dA, dX], True, True), a.reps)
        print(f"bwd  K={k} H={h}: {t * 1e3:7.1f} us  {2 * fl / t / 1e9:6.1f} TF/s  "
              f"{4 * n * (2 * h + 2 * k) / t / 1e6:6.0f} GB/s", flush=True)
        if a.check:
            ops.linear_bwd([A, X], W, dout, out, [dA, dX], True, True)
            dz = dout.double() * (out > 0)
            Xd = torch.cat([A, X], 1).double()
            dx_ref = dz @ W.double()
            e1 = float((torch.cat([dA, dX], 1) - dx_ref).abs().max() / dx_ref.abs().max())
            dw, db = ops.linear_bwd([A, X], W, dout, out, [None, None], True, True)
            dw_ref = dz.T @ Xd
            e2 = float((dw - dw_ref).abs().max() / dw_ref.abs().max())
            print(f"      check: dx rel err {e1:.1e}, dw rel err {e2:.1e}", flush=True)
        dz = torch.empty_like(out)
        t = timeit(lambda: ops.linear_bwd([A, X], W, dout, out, [dA, dX], True, True, dz_out=dz),
                   a.reps)
        print(f"bwd+dz K={k} H={h}: {t * 1e3:7.1f} us", flush=True)
        t = timeit(lambda: ops.linear_bwd([A, X], W, dout, out, [dA, dX], False, False), a.reps)
        print(f"dgrad K={k} H={h}: {t * 1e3:7.1f} us  {fl / t / 1e9:6.1f} TF/s", flush=True)
        t = timeit(lambda: ops.linear_bwd([A, X], W, dout, out, [None, None], True, True), a.reps)
        print(f"wgrad K={k} H={h}: {t * 1e3:7.1f} us  {fl / t / 1e9:6.1f} TF/s  "
              f"{4 * n * (2 * h + k) / t / 1e6:6.0f} GB/s", flush=True)
        del A, X, out, dout, dA, dX


if __name__ == "__main__":
    main()
