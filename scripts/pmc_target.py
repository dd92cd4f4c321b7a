#!/usr/bin/env python3
"""Target program for rocprofv3 --pmc passes: the cfg2 K1 forward gathers (roofline kernel) run
REPS times each, after the one-time graph build.  Prints the launch geometry so the summariser
can tell the two relations apart by grid size."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import graph, ops, synth  # noqa: E402

REPS = 5
dev = torch.device("cuda")
cfg = synth.CONFIGS["cfg2"]
g = synth.make_graph(cfg, device=dev)
eng = graph.relation_csr(g.edge_index_dict[synth.ENGAGES], cfg.num_users, cfg.num_posts)
rev = graph.relation_csr(g.edge_index_dict[synth.REV_ENGAGES], cfg.num_posts, cfg.num_users)
torch.cuda.synchronize()
info = {}
for name, csr, x in (("eng", eng, g.x_dict["user"]), ("rev", rev, g.x_dict["post"])):
    for _ in range(REPS):
        ops.gather_mean(x, csr)
    items = csr.n_dst + csr.fwd.plan.n_chunks
    info[name] = {"grid_threads": -(-items // 4) * 256, "n_dst": csr.n_dst, "n_src": csr.n_src,
                  "E": csr.num_edges, "d": cfg.dim,
                  "alg_bytes": ops.gather_bytes(csr.num_edges, csr.n_dst, cfg.dim, False)}
torch.cuda.synchronize()
print("PMC_TARGET " + json.dumps(info))
