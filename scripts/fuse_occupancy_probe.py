"""Experiment (a fused user-side gather -> K3): the user <- post K1 of cfg4
(200M edges over the 512 MB post table, 9M destination rows, d = 128) timed at the occupancy a
kernel fused with the split K3 would run at.  The K3 kernels hold ~200 VGPRs per lane and 100+
KB of LDS, so a fused kernel has 8 waves per CU; the stand-alone gather runs up to 32.  Run once
per build / env: the default library, and libhgnn_occ8.so (scripts/build_variant.py occ8
-DHGNN_GATHER_LDS=81920: two 4-wave blocks per CU), each with HGNN_G128_U=4 (8 rows in flight
per wave) and 8 (16 rows).  usage: python scripts/fuse_occupancy_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from truth_recommendation_gnn_amd import graph, ops, synth  # noqa: E402
from scripts.ic_block_bench import timed  # noqa: E402


def main():
    dev = torch.device("cuda")
    cfg = synth.CONFIGS["cfg4"]
    g = synth.make_graph(cfg, device=dev, device_gen=True)
    ei = g.edge_index_dict[synth.REV_ENGAGES]          # post -> user: users gather posts
    x = g.x_dict["post"]
    del g
    csr = graph.relation_csr(ei, cfg.num_posts, cfg.num_users)
    out = torch.empty(cfg.num_users, x.shape[1], device=dev)
    ms = timed(lambda: ops._gather(x, csr.fwd, None, False, out, False))
    E = int(ei.shape[1])
    gb = (E * (4 * 128 + 4) + cfg.num_users * 4 * 128) / 1e9
    print(json.dumps({"lib": os.environ.get("HGNN_LIB", "libhgnn.so"),
                      "rows_in_flight_per_wave": 2 * int(os.environ.get("HGNN_G128_U", "4")),
                      "ms": round(ms, 3), "GB/s": round(gb / ms * 1e3)}), flush=True)


if __name__ == "__main__":
    main()
