#!/usr/bin/env python3
"""Where the bench step and the float64 reference part (tests/f64_step.py): layer outputs, their
incoming gradients, ReLU-mask flips (fp32 output > 0 vs float64 z > 0) and the parameter-gradient
errors with the float64 masks and with the fp32 forward's masks.  Runs the HIP model layer by
layer so h1 and its gradient are visible.  usage: python scripts/f64_diag.py [cfg2|cfg4]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from truth_recommendation_gnn_amd import HeteroSAGE, graph, ops, synth  # noqa: E402
from f64_step import max_rel_err, negatives_to_coo, train_step_f64  # noqa: E402

DEV = torch.device("cuda")
RELS = [(synth.REV_ENGAGES, 1.0), (synth.ENGAGES, 1.0)]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    cfg = synth.CONFIGS[name]
    g = synth.make_graph(cfg, device=DEV)
    e = g.edge_index_dict
    pos = e[synth.ENGAGES]
    pw = synth.interaction_weights(cfg.num_posts).to(DEV)[pos[1]]
    cscale = pw.mean()
    torch.manual_seed(synth.WEIGHT_SEED)
    model = HeteroSAGE(cfg.hidden, RELS, num_layers=cfg.layers, in_channels=cfg.dim).to(DEV)
    gen = torch.Generator(device=DEV).manual_seed(synth.NEG_SEED)
    draw = ops.draw_negatives(pos, cfg.num_posts, generator=gen)
    m1 = HeteroSAGE(cfg.hidden, RELS, num_layers=1, in_channels=cfg.dim).to(DEV)
    m1.layers[0] = model.layers[0]
    m2 = HeteroSAGE(cfg.hidden, RELS, num_layers=1, in_channels=cfg.hidden).to(DEV)
    m2.layers[0] = model.layers[1]
    h1 = m1(g.x_dict, e)
    for t in h1:
        h1[t].retain_grad()
    h2 = m2(h1, e)
    loss = ops.edge_bce_loss(h2["user"], h2["post"], pos, draw, pw, neg_order="user",
                             check=False, cscale=cscale)
    loss.backward()
    got = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    params = {n: p.detach().clone() for n, p in model.named_parameters()}
    hip = {"h1_user": h1["user"].detach(), "h1_post": h1["post"].detach(),
           "h2_user": h2["user"].detach(), "h2_post": h2["post"].detach(),
           "dh1_user": h1["user"].grad, "dh1_post": h1["post"].grad}
    neg = negatives_to_coo(draw.tensor(), pos[0])
    keep = {}
    ref_loss, ref = train_step_f64(params, g.x_dict["user"], g.x_dict["post"], pos, neg,
                                   cscale.double(), keep=keep)
    rep = {"loss": [float(loss.detach()), ref_loss],
           "grad_err_f64_masks": {n: max_rel_err(got[n], ref[n]) for n in got}}
    for k, v in hip.items():
        rep[f"{k}_err"] = max_rel_err(v, keep[k])
    for l in (1, 2):
        for t in ("user", "post"):
            a, b = hip[f"h{l}_{t}"] > 0, keep[f"h{l}_{t}"] > 0
            flips = (a != b)
            rep[f"mask_flips_h{l}_{t}"] = int(flips.sum())
            if int(flips.sum()) and f"dh{l}_{t}" in keep:
                dh = keep[f"dh{l}_{t}"]
                rep[f"flip_dh_max_over_dh_max_h{l}_{t}"] = float(dh[flips].abs().max() / dh.abs().max())
    masks = [{t: hip[f"h{l}_{t}"] > 0 for t in ("user", "post")} for l in (1, 2)]
    del keep, ref
    _, ref2 = train_step_f64(params, g.x_dict["user"], g.x_dict["post"], pos, neg,
                             cscale.double(), masks=masks)
    rep["grad_err_fp32_masks"] = {n: max_rel_err(got[n], ref2[n]) for n in got}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
