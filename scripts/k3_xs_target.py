#!/usr/bin/env python3
"""rocprofv3 --pmc target: the cfg4 step's four 9M-row K3 launches, 3 times each — layer 1 user
side (forward K = 256 with the ReLU bits, its wgrad-only backward) and layer 2 (forward K = 128
with the added pre-projected rows, the backward with dgrad, dz side output and wgrad)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import ops  # noqa: E402
dev = torch.device("cuda")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 9_000_000
h = 128
A, X = torch.randn(n, 128, device=dev), torch.randn(n, 128, device=dev)
W2, W1 = torch.randn(h, 256, device=dev) * 0.1, torch.randn(h, 128, device=dev) * 0.1
b = torch.randn(h, device=dev)
add = torch.randn(n, h, device=dev)
m1, m2 = ops.relu_mask_for(n, h, True, dev), ops.relu_mask_for(n, h, True, dev)
dout = torch.randn(n, h, device=dev)
dz, dX = torch.empty(n, h, device=dev), torch.empty_like(X)
for _ in range(3):
    y1 = ops.linear_fwd([A, X], W2, b, True, mask_out=m1)
    ops.linear_bwd([A, X], W2, dout, y1, [None, None], True, True, mask=m1)
    y2 = ops.linear_fwd([X], W1, b, True, add=add, mask_out=m2)
    ops.linear_bwd([X], W1, dout, y2, [dX], True, True, dz_out=dz, mask=m2)
torch.cuda.synchronize()
# algorithmic bytes per launch of the four launches, as the bench's per-kernel timer counts them
# (one more iteration under ops.KernelTimer; scripts/pmc_k3_traffic_summarize.py divides the PMC
# bytes by these)
import json  # noqa: E402
timer = ops.KernelTimer()
ops.set_timer(timer)
y1 = ops.linear_fwd([A, X], W2, b, True, mask_out=m1)
ops.linear_bwd([A, X], W2, dout, y1, [None, None], True, True, mask=m1)
y2 = ops.linear_fwd([X], W1, b, True, add=add, mask_out=m2)
ops.linear_bwd([X], W1, dout, y2, [dX], True, True, dz_out=dz, mask=m2)
ops.set_timer(None)
torch.cuda.synchronize()
summ = timer.summary()
print("K3_ALG " + json.dumps({"n": n, "bytes": {k: v["bytes"] / v["launches"] for k, v in summ.items()}}),
      flush=True)
