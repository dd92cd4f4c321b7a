#!/usr/bin/env python3
"""rocprofv3 --pmc target: a K3 backward (dgrad + wgrad) and forward x5 each on one
destination shape.  usage: k3_target.py [n d h] (default cfg2's user side: 1M rows, two
64-wide segments -> 64; cfg4's user side: 9000000 128 128)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import ops  # noqa: E402
dev = torch.device("cuda")
n, d, h = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (1_000_000, 64, 64)
A, X = torch.randn(n, d, device=dev), torch.randn(n, d, device=dev)
W = torch.randn(h, 2 * d, device=dev) * 0.1
b = torch.randn(h, device=dev)
out = ops.linear_fwd([A, X], W, b, True)
dout = torch.randn_like(out)
dA, dX = torch.empty_like(A), torch.empty_like(X)
for _ in range(5):
    ops.linear_bwd([A, X], W, dout, out, [dA, dX], True, True)
for _ in range(5):
    ops.linear_fwd([A, X], W, b, True)
torch.cuda.synchronize()
