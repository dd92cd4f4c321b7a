"""The exact step ``bench.py`` times, end to end at the timed config, against float64.

cfg4 (the north-star graph: 9M users, 1M posts, 200M engages + the reverse relation, d = h = 128):
``HeteroSAGE`` with 2 layers as the bench builds it — the layer-2 post -> user relation
pre-projected (``ops.use_pre_projection``), the gathers over the 4.6 GB user-side tables in
source-block passes (``ops.gather_blocks``) — then ``ops.edge_bce_loss`` with a ``NegativeDraw``
(the bench's counter-based negatives, grouped by post on a side stream under the forward as the
bench does, ``presorted=``) and ``backward()``.
The loss, both layers' outputs and EVERY parameter gradient are compared with
``tests/f64_step.py`` (plain torch float64 on the GPU, aggregate-then-project, hand-written
backward) at the north_star's rtol 1e-4, read against each tensor's largest entry.  The negatives
are materialised from the same draw and mapped to COO order with torch's own stable sort.

The float64 backward takes its ReLU masks from the fp32 forward's outputs (``out > 0``, as
autograd's ReLU backward does), after those outputs are themselves checked against float64: an
element whose pre-activation lies within fp32 rounding of 0 can be 0 in fp32 and positive in
float64, and one such element in a Zipf-hot post row moves a layer-1 weight gradient by ~1e-4 of
its max (cfg2: one flip among 6.4M post elements; ``scripts/f64_diag.py``).  The flips are
counted and bounded.  cfg2 runs the same check at the smaller graph, where no gather is
source-blocked.
Reference step: train_gnn.py:242-285 (forward 254, loss 259-281, backward 283).
"""
import gc

import pytest
import torch

from truth_recommendation_gnn_amd import HeteroSAGE, graph, ops, synth

from f64_step import max_rel_err, negatives_to_coo, train_step_f64

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
RELS = [(synth.REV_ENGAGES, 1.0), (synth.ENGAGES, 1.0)]
RTOL = 1e-4


def _free():
    graph.CSR_CACHE.clear()
    gc.collect()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name", ["cfg2", "cfg4"])
def test_bench_step_matches_float64(name):
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

    timer = ops.KernelTimer()            # only to see which launches the step made
    ops.set_timer(timer)
    try:
        # as the bench: the negatives grouped by post on a side stream under the forward
        main, side = torch.cuda.current_stream(DEV), torch.cuda.Stream(DEV)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            pre = ops.presort_negatives(cfg.num_users, cfg.num_posts, pos, draw, "user")
        pre.rowptr.record_stream(main)
        pre.users.record_stream(main)
        out = model(g.x_dict, e)
        main.wait_stream(side)
        loss = ops.edge_bce_loss(out["user"], out["post"], pos, draw, pw, neg_order="user",
                                 check=False, cscale=cscale, presorted=pre)
        loss.backward()
    finally:
        ops.set_timer(None)
    names = set(timer.summary())
    got_loss = float(loss.detach())
    got = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    params = {n: p.detach().clone() for n, p in model.named_parameters()}
    h2 = {t: out[t].detach() for t in ("user", "post")}
    # the layer-1 output the fused step computed internally: layer 1 alone, and layer 2 on it
    # must give the fused forward's output bit for bit (grad mode on, as in the step: it decides
    # where the pre-projection applies)
    m1 = HeteroSAGE(cfg.hidden, RELS, num_layers=1, in_channels=cfg.dim).to(DEV)
    m1.layers[0] = model.layers[0]
    m2 = HeteroSAGE(cfg.hidden, RELS, num_layers=1, in_channels=cfg.hidden).to(DEV)
    m2.layers[0] = model.layers[1]
    h1 = m1(g.x_dict, e)
    again = m2(h1, e)
    for t in ("user", "post"):
        assert torch.equal(again[t].detach(), h2[t])
    h1 = {t: v.detach() for t, v in h1.items()}
    del again, m1, m2
    if name == "cfg4":
        # the bench's composition was taken: layer 2's user update is a K = 128 GEMM with the
        # gathered projected post rows added (pre-projection), and the post <- user gathers over
        # the 4.6 GB tables ran source-blocked
        assert f"linear_fwd[{cfg.num_users}x{cfg.hidden}->{cfg.hidden}]" in names, sorted(names)
        assert ops.gather_blocks(g.x_dict["user"]) > 1
        csr = graph.relation_csr(pos, cfg.num_users, cfg.num_posts)
        assert any(k[0] == "fwd" and k[1] > 1 for k in csr.__dict__.get("_blocks", {}))
    neg = negatives_to_coo(draw.tensor(), pos[0])
    del out, loss, timer
    _free()

    masks = [{t: h1[t] > 0 for t in ("user", "post")}, {t: h2[t] > 0 for t in ("user", "post")}]
    keep = {}
    ref_loss, ref = train_step_f64(params, g.x_dict["user"], g.x_dict["post"], pos, neg,
                                   cscale.double(), masks=masks, keep=keep)
    fwd_errs, flips = {}, {}
    for l, h in ((1, h1), (2, h2)):
        for t in ("user", "post"):
            r = keep[f"h{l}_{t}"]
            fwd_errs[f"h{l}_{t}"] = max_rel_err(h[t], r)
            flips[f"h{l}_{t}"] = int(((h[t] > 0) != (r > 0)).sum())
    errs = {n: max_rel_err(got[n], ref[n]) for n in got}
    assert set(ref) == set(got)
    assert abs(got_loss - ref_loss) <= RTOL * abs(ref_loss), (got_loss, ref_loss)
    assert max(fwd_errs.values()) < RTOL, fwd_errs
    # sign disagreements only where the forward's own tolerance reaches 0: both values of every
    # flipped element within 1e-4 of the output's max
    for l, h in ((1, h1), (2, h2)):
        for t in ("user", "post"):
            r = keep[f"h{l}_{t}"]
            f = (h[t] > 0) != (r > 0)
            if bool(f.any()):
                worst = max(float(h[t][f].abs().max()), float(r[f].abs().max()))
                assert worst <= RTOL * float(r.abs().max()), (l, t, worst)
    assert max(errs.values()) < RTOL, errs
    print(f"{name}: loss {got_loss:.8f} vs {ref_loss:.8f}; forward max rel err "
          f"{max(fwd_errs.values()):.2e}; mask flips {flips}; grad max rel err "
          f"{max(errs.values()):.2e}")
    del ref, keep, g, e, pos, pw, neg, h1, h2, masks
    _free()
