#!/usr/bin/env python3
"""rocprofv3 target: one cfg2-scale evaluation (10% of the engages as test edges)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import metrics, synth  # noqa: E402
dev = torch.device("cuda")
cfg = synth.CONFIGS["cfg2"]
g = synth.make_graph(cfg, device=dev)
U, P = g.x_dict["user"], g.x_dict["post"]
te = g.edge_index_dict[synth.ENGAGES][:, ::10].clone()
te[1] += cfg.num_users
metrics.evaluate(te, U, P, K=10)
torch.cuda.synchronize()
