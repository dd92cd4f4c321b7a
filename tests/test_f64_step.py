"""Pins the float64 step reference (tests/f64_step.py) that the cfg2/cfg4 end-to-end GPU tests
compare the bench step with: on small graphs on the CPU it must equal the oracle's autograd
(oracle/sage_ref.py, PyG's op pattern) run in float64 — loss and every parameter gradient."""
import torch

from oracle import sage_ref
from truth_recommendation_gnn_amd import synth

from f64_step import max_rel_err, negatives_to_coo, train_step_f64

RELS = [(synth.REV_ENGAGES, 1.0), (synth.ENGAGES, 1.0)]


def _names(cfg, layers):
    out = []
    for l in range(layers):
        cin = cfg.dim if l == 0 else cfg.hidden
        for et, _ in RELS:
            p = f"layers.{l}.{'__'.join(et)}"
            out += [(f"{p}.lin_l.weight", (cfg.hidden, cin)), (f"{p}.lin_l.bias", (cfg.hidden,)),
                    (f"{p}.lin_r.weight", (cfg.hidden, cin))]
    return out


def _check(cfg, layers):
    g = synth.make_graph(cfg)
    pos = g.edge_index_dict[synth.ENGAGES]
    neg = synth.negative_posts(cfg.num_posts, pos.shape[1])
    pw = synth.interaction_weights(cfg.num_posts)[pos[1]]
    params = {k: v.double() for k, v in sage_ref.init_params(_names(cfg, layers)).items()}
    x = {k: v.double() for k, v in g.x_dict.items()}
    P = {k: v.clone().requires_grad_() for k, v in params.items()}
    out = sage_ref.hetero_sage(P, x, g.edge_index_dict, RELS, layers)
    loss = sage_ref.link_loss(out["user"], out["post"], pos, neg, pw.double())
    loss.backward()
    got_loss, got = train_step_f64(params, g.x_dict["user"], g.x_dict["post"], pos, neg,
                                   pw.double().mean(), layers=layers)
    assert abs(got_loss - float(loss.detach())) <= 1e-12 * abs(float(loss.detach()))
    assert set(got) == set(P)
    for k, p in P.items():
        assert max_rel_err(got[k], p.grad) < 1e-10, k


def test_f64_step_equals_oracle_autograd_two_layers():
    cfg = synth.dataclasses.replace(synth.scaled("cfg2", 0.0005), dim=16, hidden=12)
    _check(cfg, 2)


def test_f64_step_equals_oracle_autograd_three_layers_zero_degree_rows():
    # 50 posts over 40 edges: many posts without an engager (zero-degree rows of the mean)
    cfg = synth.dataclasses.replace(synth.scaled("cfg2", 0.0005), num_posts=50, num_engages=40,
                                    dim=8, hidden=8)
    _check(cfg, 3)


def test_negatives_to_coo_inverts_the_user_grouping():
    users = torch.tensor([3, 1, 3, 0, 1, 3])
    coo = torch.tensor([10, 11, 12, 13, 14, 15])
    order = torch.argsort(users, stable=True)        # the user-grouped positions
    assert torch.equal(negatives_to_coo(coo[order], users), coo)
