"""float64 reference of one training step of the bench's model — TEST ONLY.

The step ``bench.py`` times at N = 1 (and, sharded, at N > 1): the 2-layer relation-weighted
hetero SAGE (``HeteroSAGE`` over ``rev_engages`` post -> user and ``engages`` user -> post, weights
1.0, ReLU after each layer — the reference layer ``train_gnn.py:166-200`` stacked twice), the
reference link loss (``train_gnn.py:259-281``: BCE-with-logits, mean reduction, so the per-edge
interaction weights collapse to their mean) and its full backward (``train_gnn.py:283``).

Written in plain torch float64 on the GPU, with no hgnn call and none of the build's algebra: the
means are aggregated first and projected afterwards (the reference's order, not the build's
pre-projection), every sum over edges is an ``index_add_`` over the COO edge list in edge chunks
(an autograd ``index_select`` over 200M edges would hold ~205 GB), and the backward is written out
by hand.  It is independent of the kernels it checks; the fp32 / float64 gap it leaves is the
north_star's tolerance (rtol 1e-4).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn.functional as F

CHUNK = 1 << 22                 # edges per float64 chunk (4M x 128 x 8 B = 4 GB per temporary)
ROWS = 1 << 21                  # rows per float64 GEMM chunk

REL_USER = "post__rev_engages__user"     # post -> user: the user-side update
REL_POST = "user__engages__post"         # user -> post: the post-side update


def _seg_mean(dst, src, table, n_dst, inv_deg):
    """float64 [n_dst, d]: mean over edges e (dst[e] = i) of table[src[e]] (0 for no edge)."""
    out = torch.zeros(n_dst, table.shape[1], dtype=torch.float64, device=table.device)
    for s in range(0, dst.numel(), CHUNK):
        out.index_add_(0, dst[s:s + CHUNK], table[src[s:s + CHUNK]].double())
    return out.mul_(inv_deg[:, None])


def _seg_scatter(src, dst, g, n_src, inv_deg):
    """Transpose of _seg_mean: float64 [n_src, d], row j = sum_{e: src[e] = j} g[dst[e]] / deg."""
    out = torch.zeros(n_src, g.shape[1], dtype=torch.float64, device=g.device)
    for s in range(0, dst.numel(), CHUNK):
        d = dst[s:s + CHUNK]
        out.index_add_(0, src[s:s + CHUNK], g[d] * inv_deg[d][:, None])
    return out


def _lin(x, w):
    """x @ w^T in float64, x converted per row chunk (x may be an fp32 input table)."""
    out = torch.empty(x.shape[0], w.shape[0], dtype=torch.float64, device=x.device)
    for s in range(0, x.shape[0], ROWS):
        out[s:s + ROWS] = x[s:s + ROWS].double() @ w.T
    return out


def _tmm(a, b):
    """a^T @ b over all rows (a float64, b possibly fp32), accumulated in float64."""
    acc = torch.zeros(a.shape[1], b.shape[1], dtype=torch.float64, device=a.device)
    for s in range(0, a.shape[0], ROWS):
        acc += a[s:s + ROWS].T @ b[s:s + ROWS].double()
    return acc


def train_step_f64(params: Dict[str, torch.Tensor], x_user: torch.Tensor, x_post: torch.Tensor,
                   pos: torch.Tensor, neg: torch.Tensor, cscale, layers: int = 2,
                   masks=None, keep=None) -> Tuple[float, Dict[str, torch.Tensor]]:
    """(loss, {parameter name: float64 gradient}) of one step.

    ``pos``: the engages edges [2, E] (user, post) in COO order; ``neg``: one negative post per
    COO edge (train_gnn.py:272); ``cscale``: mean of the interaction weights of the positive
    edges (train_gnn.py:280 collapses the per-edge weights to it).  ``masks`` (optional):
    ``masks[l][type]`` replaces layer l's ReLU mask ``z > 0`` (diagnostics); ``keep`` (optional
    dict) receives the layer outputs ``h{l}_{type}`` and their incoming gradients
    ``dh{l}_{type}`` (before the mask)."""
    dev = x_user.device
    W = {k: v.detach().to(dev, torch.float64) for k, v in params.items()}
    n_u, n_p = x_user.shape[0], x_post.shape[0]
    u_idx, p_idx = pos[0].long(), pos[1].long()
    neg = neg.long()
    E = u_idx.numel()
    inv_u = 1.0 / torch.bincount(u_idx, minlength=n_u).double().clamp(min=1)
    inv_p = 1.0 / torch.bincount(p_idx, minlength=n_p).double().clamp(min=1)

    # forward (train_gnn.py:177-198 per layer): aggregate, then project
    h = {"user": x_user, "post": x_post}
    saved = []
    for l in range(layers):
        ru, rp = f"layers.{l}.{REL_USER}", f"layers.{l}.{REL_POST}"
        agg_u = _seg_mean(u_idx, p_idx, h["post"], n_u, inv_u)      # rev_engages: post -> user
        agg_p = _seg_mean(p_idx, u_idx, h["user"], n_p, inv_p)      # engages: user -> post
        z_u = _lin(agg_u, W[f"{ru}.lin_l.weight"])
        z_u += W[f"{ru}.lin_l.bias"]
        z_u += _lin(h["user"], W[f"{ru}.lin_r.weight"])
        z_p = _lin(agg_p, W[f"{rp}.lin_l.weight"])
        z_p += W[f"{rp}.lin_l.bias"]
        z_p += _lin(h["post"], W[f"{rp}.lin_r.weight"])
        saved.append((h, agg_u, agg_p))
        h = {"user": z_u.relu_(), "post": z_p.relu_()}
        if keep is not None:
            keep[f"h{l + 1}_user"], keep[f"h{l + 1}_post"] = h["user"], h["post"]
    Ue, Pe = h["user"], h["post"]

    # the loss and dL/dU, dL/dP (train_gnn.py:259-281)
    c = float(cscale)
    lp = torch.zeros((), dtype=torch.float64, device=dev)
    ln = torch.zeros((), dtype=torch.float64, device=dev)
    dU = torch.zeros_like(Ue)
    dP = torch.zeros_like(Pe)
    for s in range(0, E, CHUNK):
        ui, pi, ni = u_idx[s:s + CHUNK], p_idx[s:s + CHUNK], neg[s:s + CHUNK]
        u = Ue[ui]
        pp = Pe[pi]
        sp = (u * pp).sum(1)
        lp += F.softplus(-sp).sum()
        gp = (-c / E) * torch.sigmoid(-sp)
        nn_ = Pe[ni]
        sn = (u * nn_).sum(1)
        ln += F.softplus(sn).sum()
        gn = torch.sigmoid(sn) / E
        dU.index_add_(0, ui, pp.mul_(gp[:, None]).add_(nn_.mul_(gn[:, None])))
        dP.index_add_(0, pi, u * gp[:, None])
        dP.index_add_(0, ni, u.mul_(gn[:, None]))
        del u, pp, nn_
    loss = float(c * lp / E + ln / E)

    # backward, layer by layer
    grads: Dict[str, torch.Tensor] = {}
    dh = {"user": dU, "post": dP}
    out = h
    for l in reversed(range(layers)):
        h_in, agg_u, agg_p = saved[l]
        ru, rp = f"layers.{l}.{REL_USER}", f"layers.{l}.{REL_POST}"
        if keep is not None:
            keep[f"dh{l + 1}_user"] = dh["user"].clone()
            keep[f"dh{l + 1}_post"] = dh["post"].clone()
        mk = masks[l] if masks is not None else {t: out[t] > 0 for t in ("user", "post")}
        dz_u = dh["user"].mul_(mk["user"])               # ReLU's backward from its output
        dz_p = dh["post"].mul_(mk["post"])
        grads[f"{ru}.lin_l.weight"] = _tmm(dz_u, agg_u)
        grads[f"{ru}.lin_l.bias"] = dz_u.sum(0)
        grads[f"{ru}.lin_r.weight"] = _tmm(dz_u, h_in["user"])
        grads[f"{rp}.lin_l.weight"] = _tmm(dz_p, agg_p)
        grads[f"{rp}.lin_l.bias"] = dz_p.sum(0)
        grads[f"{rp}.lin_r.weight"] = _tmm(dz_p, h_in["post"])
        if l == 0:
            break
        del agg_u, agg_p
        saved[l] = None
        # d h_in: the root terms plus the mean scatters' transposes
        d_post = _seg_scatter(p_idx, u_idx, dz_u @ W[f"{ru}.lin_l.weight"], n_p, inv_u)
        d_post += dz_p @ W[f"{rp}.lin_r.weight"]
        d_user = _seg_scatter(u_idx, p_idx, dz_p @ W[f"{rp}.lin_l.weight"], n_u, inv_p)
        d_user += _lin(dz_u, W[f"{ru}.lin_r.weight"].T)
        del dz_u, dz_p
        dh = {"user": d_user, "post": d_post}
        out = h_in
    return loss, grads


def negatives_to_coo(neg_user_order: torch.Tensor, users: torch.Tensor) -> torch.Tensor:
    """Negatives drawn in the user-grouped order (``ops.draw_negatives`` / ``sample_negatives``:
    position i of the edges grouped by user, COO order within a user) -> per COO edge.  The
    grouping is recomputed here with torch's stable sort, not taken from the build's CSC."""
    order = torch.argsort(users, stable=True)
    out = torch.empty(users.numel(), dtype=torch.int64, device=users.device)
    out[order] = neg_user_order.long()
    return out


def max_rel_err(got: torch.Tensor, ref: torch.Tensor) -> float:
    """max |got - ref| / max |ref| (the north_star's rtol 1e-4 read against the tensor's max)."""
    return float((got.double() - ref.double()).abs().max()) / max(float(ref.abs().max()), 1e-30)
