#!/usr/bin/env python3
"""K3 at the cfg4 step's shapes (HIP events), each result checked against float64 torch: the
kernel family comes from the environment (HGNN_K3_X6=0: the f32-input kernels instead of the
bf16x6 split), read once per process, so run one process per family.

  python scripts/k3_xs_bench.py [--rows 9000000] [--post-rows 1000000] [--reps 10]

Bytes per launch are the algorithmic HBM bytes of DESIGN.md §5 (inputs read once, outputs
written once); frac = GB/s / 8000."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import ops  # noqa: E402


def timeit(fn, reps):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def rel(a, b):
    b = b.to(torch.float64)
    return float((a.to(torch.float64) - b).abs().max() / b.abs().max().clamp_min(1e-30))


def case(name, n, ks, relu, add_on, mask_on, bwd_dx, bwd_w, dz_on, reps, dev, g, out):
    h = 128
    segs = [torch.randn(n, k, device=dev, generator=g) for k in ks]
    w = torch.randn(h, sum(ks), device=dev, generator=g) * 0.1
    b = torch.randn(h, device=dev, generator=g)
    add = torch.randn(n, h, device=dev, generator=g) if add_on else None
    mk = ops.relu_mask_for(n, h, relu, dev) if mask_on else None
    y = ops.linear_fwd(segs, w, b, relu, add=add, mask_out=mk)
    # float64 reference in row chunks
    err_f, mask_ok = 0.0, True
    for r0 in range(0, n, 1 << 21):
        r1 = min(n, r0 + (1 << 21))
        x = torch.cat([s[r0:r1] for s in segs], 1).double()
        ref = x @ w.double().t() + b.double()
        if add is not None:
            ref += add[r0:r1].double()
        if relu:
            ref.relu_()
        err_f = max(err_f, rel(y[r0:r1], ref))
        if mk is not None:   # bit 4c+e of word 4 row + g <-> column 16 c + 4 g + e
            pos = (y[r0:r1] > 0).view(-1, 8, 4, 4).permute(0, 2, 1, 3).reshape(-1, 4, 32)
            words = (pos.to(torch.int64) << torch.arange(32, device=dev)).sum(-1)
            mask_ok &= bool(torch.equal(words.to(torch.int64) & 0xFFFFFFFF,
                                        mk[r0:r1].to(torch.int64) & 0xFFFFFFFF))
    del x, ref
    ms = timeit(lambda: ops.linear_fwd(segs, w, b, relu, add=add, mask_out=mk), reps)
    nb = 4 * n * (sum(ks) + h) + (4 * n * h if add_on else 0) + (16 * n if mk is not None else 0)
    rec = {"case": name, "fwd_ms": round(ms, 3), "fwd_GBs": round(nb / ms / 1e6, 1),
           "fwd_frac": round(nb / ms / 1e6 / 8000, 3), "fwd_rel_err": float(f"{err_f:.2e}"),
           "mask_bits_ok": mask_ok if mk is not None else None}
    if bwd_dx or bwd_w:
        dout = torch.randn(n, h, device=dev, generator=g)
        dxs = [torch.empty_like(s) if (bwd_dx and si == len(segs) - 1) else None
               for si, s in enumerate(segs)]
        dz = torch.empty(n, h, device=dev) if dz_on else None
        res = ops.linear_bwd(segs, w, dout, y if relu else None, dxs, bwd_w, bwd_w, dz_out=dz,
                             mask=mk)
        dw, db = res[0], res[1]
        dzr = (dout * (y > 0)) if relu else dout
        e = {}
        if dz is not None:
            e["dz"] = rel(dz, dzr)
        if bwd_dx:
            k0 = sum(ks[:-1])
            e["dx"] = max(rel(dxs[-1][r0:r0 + (1 << 21)],
                              dzr[r0:r0 + (1 << 21)].double() @ w[:, k0:].double())
                          for r0 in range(0, n, 1 << 21))
        if bwd_w:
            dwr = torch.zeros(h, sum(ks), dtype=torch.float64, device=dev)
            for r0 in range(0, n, 1 << 21):
                x = torch.cat([s[r0:r0 + (1 << 21)] for s in segs], 1).double()
                dwr += dzr[r0:r0 + (1 << 21)].double().t() @ x
            e["dw"] = rel(dw, dwr)
            e["db"] = rel(db, dzr.double().sum(0))
        ms_b = timeit(lambda: ops.linear_bwd(segs, w, dout, y if relu else None, dxs, bwd_w, bwd_w,
                                             dz_out=dz, mask=mk), reps)
        nbb = 4 * n * (h + sum(ks)) + (16 * n if mk is not None else 0) + \
            (4 * n * ks[-1] if bwd_dx else 0) + (4 * n * h if dz_on else 0)
        rec.update({"bwd_ms": round(ms_b, 3), "bwd_GBs": round(nbb / ms_b / 1e6, 1),
                    "bwd_frac": round(nbb / ms_b / 1e6 / 8000, 3),
                    "bwd_rel_err": {k: float(f"{v:.2e}") for k, v in e.items()}})
    rec["family"] = "f32" if os.environ.get("HGNN_K3_X6") == "0" else "bf16x6 split-once"
    out.append(rec)
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=9_000_000)
    ap.add_argument("--post-rows", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    out = []
    U, P = a.rows, a.post_rows
    cases = [
        # name, n, ks, relu, add, mask, bwd dx, bwd w, dz_out
        ("user_l1 fwd K256 + bwd wgrad", U, [128, 128], True, False, True, False, True, False),
        ("user_l2 fwd K128+add + bwd dx/dz/wgrad", U, [128], True, True, True, True, True, True),
        ("post_l1 fwd K256 + bwd wgrad", P, [128, 128], True, False, True, False, True, False),
        ("post_l2 fwd K256 + bwd dx/wgrad", P, [128, 128], True, False, True, True, True, False),
        ("preproj fwd K128 (no relu) + bwd dx/wgrad", P, [128], False, False, False, True, True,
         False),
    ]
    for c in cases:
        if a.only and a.only not in c[0]:
            continue
        case(*c, a.reps, dev, g, out)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
