#!/usr/bin/env python3
"""Where a split-once K3 forward iteration spends its time, from in-kernel s_memtime stamps (a
diagnostic build: `python scripts/build_variant.py stamps -DHGNN_XS_STAMPS=1 --only linear_xs`,
run with HGNN_LIB=libhgnn_stamps.so).  Lane 0 of every wave of blocks 0-63 stamps 7 points of
iterations 40-47: 0 top, 1 after the late waves' split, 2 after the output stores + the prefetch
issue, 3 after the MFMA sweep is issued, 4 after the epilogue, 5 after the early waves' split,
6 after the barrier (8 / 9: after an explicit wait for the loads before the late / early split).  The backward kernel stamps 8 points: top, after the late waves'
put, after the memory issue, after the dgrad sweep, after the wgrad sweep, after the dX stores,
after the early waves' put, after the barrier.  Prints the mean cycles of each phase for waves
0-3 (early) and 4-7 (late) per shape, as one JSON line each.
usage: HGNN_LIB=libhgnn_stamps.so python scripts/k3_stamps.py [rows]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import _native as N, ops  # noqa: E402

BLOCKS, WAVES, ITERS, PTS = 64, 8, 8, 12
NAMES = {"fwd": ["late_split", "stores+issue", "sweep_issue", "epilogue", "early_split", "barrier"],
         "bwd": ["late_put", "vmem_issue", "dgrad_sweep", "wgrad_sweep", "dx_stores", "early_put",
                 "barrier"]}


def read():
    lib = N.lib()
    f = lib.hgnn_debug_xs_stamps
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(BLOCKS * WAVES * ITERS * PTS, dtype=np.uint64)
    torch.cuda.synchronize()
    n = f(buf.ctypes.data, buf.size)
    assert n == buf.size, n
    return buf.reshape(BLOCKS, WAVES, ITERS, PTS).astype(np.int64)


def main():
    dev = torch.device("cuda")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 9_000_000
    h = 128
    g = torch.Generator(device=dev).manual_seed(0)
    A, X = torch.randn(n, 128, device=dev, generator=g), torch.randn(n, 128, device=dev, generator=g)
    W2, W1 = torch.randn(h, 256, device=dev, generator=g) * 0.1, torch.randn(h, 128, device=dev, generator=g) * 0.1
    b = torch.randn(h, device=dev, generator=g)
    add = torch.randn(n, h, device=dev, generator=g)
    m = ops.relu_mask_for(n, h, True, dev)
    y1 = ops.linear_fwd([A, X], W2, b, True, mask_out=m)
    m2 = ops.relu_mask_for(n, h, True, dev)
    y2 = ops.linear_fwd([X], W1, b, True, add=add, mask_out=m2)
    dout = torch.randn(n, h, device=dev, generator=g)
    dz, dX = torch.empty(n, h, device=dev), torch.empty_like(X)
    cases = (("fwd K256", "fwd", lambda: ops.linear_fwd([A, X], W2, b, True, mask_out=m)),
             ("fwd K128+add", "fwd",
              lambda: ops.linear_fwd([X], W1, b, True, add=add, mask_out=m2)),
             ("bwd K256 wgrad", "bwd",
              lambda: ops.linear_bwd([A, X], W2, dout, y1, [None, None], True, True, mask=m)),
             ("bwd K128 dx+dz+wgrad", "bwd",
              lambda: ops.linear_bwd([X], W1, dout, y2, [dX], True, True, dz_out=dz, mask=m2)))
    for name, kind, fn in cases:
        for _ in range(3):
            fn()
        s = read()
        names = NAMES[kind]
        npts = len(names) + 1
        d = np.diff(s[..., :npts], axis=-1)
        tot = s[..., npts - 1] - s[..., 0]
        rec = {"case": name}
        for lo, hi, tag in ((0, 4, "early"), (4, 8, "late")):
            ph = d[:, lo:hi].reshape(-1, npts - 1).mean(0)
            rec[tag] = {k: round(float(v), 1) for k, v in zip(names, ph)}
            rec[tag]["iteration"] = round(float(tot[:, lo:hi].mean()), 1)
        # the split's wait for its loads (points 8 / 9, an explicit vmcnt(0) before the split)
        sp = len(names) - 2   # the point before the early split
        late_w = (s[:, 4:8, :, 8] - s[:, 4:8, :, 0]).mean()
        early_w = (s[:, 0:4, :, 9] - s[:, 0:4, :, sp]).mean()
        rec["late"]["split_load_wait"] = round(float(late_w), 1)
        rec["early"]["split_load_wait"] = round(float(early_w), 1)
        if kind == "bwd":   # the late put: dz part (8 -> 10), X part (10 -> 11)
            rec["late"]["put_dz"] = round(float((s[:, 4:8, :, 10] - s[:, 4:8, :, 8]).mean()), 1)
            rec["late"]["put_x"] = round(float((s[:, 4:8, :, 11] - s[:, 4:8, :, 10]).mean()), 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
