"""CPU ORACLE — test infrastructure only, never the product path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
module, and only as the checker (or, for the CPU baseline, as the thing timed on host cores).
The shipped path (``truth_recommendation_gnn_amd``) never imports it and fails loudly when its
HIP library is missing.

What it restates (plain PyTorch on CPU, the same op pattern PyG uses — materialised
``index_select`` gather, ``scatter_reduce(mean)``, ``addmm``):

* PyG ``SAGEConv((-1,-1), h)`` with its defaults (aggr='mean', root_weight=True, normalize=False,
  bias on ``lin_l`` only), as called at ``train_gnn.py:158-160,177-198``:
  ``out = lin_l(mean_{(j->i)} x_src[j]) + lin_r(x_dst[i])``; flow source_to_target
  (row 0 = source, row 1 = destination); duplicate edges count with multiplicity; a destination
  with no in-edges aggregates to exactly 0.
* ``WeightedRGCN.forward`` (``train_gnn.py:166-200``): user = relu(1.0*direct + 0.75*social),
  post = relu(post_update); and the 3-message variant of ``test_gnn.py:136-168`` (weights
  1.75 / 0.7 / 0.3 at ``test_gnn.py:132-134``).
* the training loss (``train_gnn.py:259-281``) including its scalar-collapse quirk:
  ``BCEWithLogitsLoss()`` reduces to a scalar, so ``(pos_weights * pos_loss).mean()`` equals
  ``mean(pos_weights) * pos_loss``.
* ``HeteroSAGE``: the same relation-weighted SAGE layer stacked ``L`` times (BASELINE configs
  2-5 are 2-layer), ReLU after every layer as in the reference layer.

PARITY STATUS: **parity unpinned** against the reference itself.  The reference ships no test,
golden vector or fixture for this path, importing its scripts was denied in this
environment, and the library that holds the arithmetic (torch_geometric) is not
installed and not vendored.  This restatement is instead pinned by an independent float64
dense-adjacency formulation (``oracle/dense_ref.py``) and by the properties in
``tests/test_oracle.py``; the golden fixtures under ``tests/golden/`` are its outputs.
"""
from __future__ import annotations

from typing import Dict, Iterable, Mapping, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

EdgeType = Tuple[str, str, str]


def mean_aggregate(x_src: torch.Tensor, edge_index: torch.Tensor, n_dst: int) -> torch.Tensor:
    """PyG ``propagate`` with aggr='mean': gather ``x_src[src]`` ([E,d], materialised) then
    ``scatter_reduce(..., 'mean', include_self=False)`` by ``dst`` into zeros (empty rows = 0)."""
    src, dst = edge_index[0], edge_index[1]
    d = x_src.shape[1]
    out = torch.zeros(n_dst, d, dtype=x_src.dtype)
    if src.numel() == 0:
        return out
    msg = x_src.index_select(0, src)
    return out.scatter_reduce(0, dst.view(-1, 1).expand(-1, d), msg, reduce="mean",
                              include_self=False)


def sage_conv(x_src: torch.Tensor, x_dst: torch.Tensor, edge_index: torch.Tensor,
              w_l: torch.Tensor, b_l: Optional[torch.Tensor], w_r: torch.Tensor) -> torch.Tensor:
    """``SAGEConv((x_src, x_dst), edge_index)``: ``lin_l(aggr) + lin_r(x_dst)``."""
    aggr = mean_aggregate(x_src, edge_index, x_dst.shape[0])
    out = F.linear(aggr, w_l, b_l)
    return out + F.linear(x_dst, w_r)


def _conv_params(params: Mapping[str, torch.Tensor], prefix: str):
    return (params[f"{prefix}.lin_l.weight"], params.get(f"{prefix}.lin_l.bias"),
            params[f"{prefix}.lin_r.weight"])


# (module name, edge type, weight) per destination, as train_gnn.py:177-198 wires them.
TRAIN_LAYOUT = {
    "user": [("msg_direct", ("post", "rev_engages", "user"), 1.0),
             ("msg_social", ("user", "social", "user"), 0.75)],
    "post": [("post_update", ("user", "engages", "post"), 1.0)],
}
# test_gnn.py:126-168 (3-message variant; followed_by is usually empty there)
TEST_LAYOUT = {
    "user": [("msg_direct", ("post", "rev_engages", "user"), 1.75),
             ("msg_author", ("post", "followed_by", "user"), 0.7),
             ("msg_social", ("user", "social", "user"), 0.3)],
    "post": [("post_update", ("user", "engages", "post"), 1.0)],
}


def weighted_rgcn(params: Mapping[str, torch.Tensor], x_dict: Mapping[str, torch.Tensor],
                  edge_index_dict: Mapping[EdgeType, torch.Tensor],
                  layout=TRAIN_LAYOUT) -> Dict[str, torch.Tensor]:
    """``WeightedRGCN.forward`` (train_gnn.py:166-200): per destination type, the weighted sum
    of its SAGE messages in the reference's order, then ReLU."""
    out = {}
    for dst_t, msgs in layout.items():
        acc = None
        for name, et, w in msgs:
            src_t = et[0]
            m = sage_conv(x_dict[src_t], x_dict[dst_t], edge_index_dict[et],
                          *_conv_params(params, name))
            term = w * m
            acc = term if acc is None else acc + term
        out[dst_t] = F.relu(acc)
    return out


def hetero_sage(params: Mapping[str, torch.Tensor], x_dict: Mapping[str, torch.Tensor],
                edge_index_dict: Mapping[EdgeType, torch.Tensor],
                relations: Sequence[Tuple[EdgeType, float]], num_layers: int
                ) -> Dict[str, torch.Tensor]:
    """L stacked relation-weighted SAGE layers.  Parameter names
    ``layers.{l}.{src}__{rel}__{dst}.lin_{l,r}.*``; node types with no incoming relation keep
    their input unchanged."""
    h = dict(x_dict)
    for layer in range(num_layers):
        nxt = {}
        for dst_t in sorted({et[2] for et, _ in relations}):
            acc = None
            for et, w in relations:
                if et[2] != dst_t:
                    continue
                name = f"layers.{layer}.{'__'.join(et)}"
                m = sage_conv(h[et[0]], h[dst_t], edge_index_dict[et], *_conv_params(params, name))
                acc = w * m if acc is None else acc + w * m
            nxt[dst_t] = F.relu(acc)
        for t in h:
            nxt.setdefault(t, h[t])
        h = nxt
    return h


def hetero_sage_blocks(params: Mapping[str, torch.Tensor], x_in: Mapping[str, torch.Tensor],
                       blocks: Sequence[Tuple[Mapping[EdgeType, torch.Tensor], Mapping[str, int]]],
                       relations: Sequence[Tuple[EdgeType, float]]) -> Dict[str, torch.Tensor]:
    """``hetero_sage`` on sampled blocks (PyG NeighborLoader's layer-wise bipartite graphs):
    block l is (local ``edge_index_dict``, ``n_dst`` per type); its destinations are the first
    ``n_dst[t]`` of its source nodes of type ``t``, so the root term reads that prefix.  Types with
    no relation into them keep that prefix unchanged."""
    h = dict(x_in)
    for layer, (eid, n_dst) in enumerate(blocks):
        nxt = {}
        for dst_t, nd in n_dst.items():
            acc = None
            for et, w in relations:
                if et[2] != dst_t or et not in eid:
                    continue
                name = f"layers.{layer}.{'__'.join(et)}"
                m = sage_conv(h[et[0]], h[dst_t][:nd], eid[et], *_conv_params(params, name))
                acc = w * m if acc is None else acc + w * m
            nxt[dst_t] = F.relu(acc) if acc is not None else h[dst_t][:nd]
        h = nxt
    return h


def link_loss(user_emb: torch.Tensor, post_emb: torch.Tensor, pos_edges: torch.Tensor,
              neg_p: torch.Tensor, pos_weights: torch.Tensor) -> torch.Tensor:
    """train_gnn.py:259-281.  ``pos_weights`` is the per-positive-edge interaction weight
    (``interaction_type_tensor[pos_p + num_users]``); ``neg_p`` is injected."""
    pos_u, pos_p = pos_edges[0], pos_edges[1]
    pos_scores = (user_emb[pos_u] * post_emb[pos_p]).sum(dim=1)
    neg_scores = (user_emb[pos_u] * post_emb[neg_p]).sum(dim=1)
    crit = torch.nn.BCEWithLogitsLoss()
    pos_loss = crit(pos_scores, torch.ones_like(pos_scores))
    neg_loss = crit(neg_scores, torch.zeros_like(neg_scores))
    return (pos_weights * pos_loss).mean() + neg_loss


def train_step_grads(params: Dict[str, torch.Tensor], forward, pos_edges, neg_p, pos_weights):
    """One fwd + loss + bwd; returns (outputs, loss, {name: grad})."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    out = forward(leaves)
    loss = link_loss(out["user"], out["post"], pos_edges, neg_p, pos_weights)
    loss.backward()
    return ({k: v.detach() for k, v in out.items()}, loss.detach(),
            {k: v.grad.detach() if v.grad is not None else torch.zeros_like(v)
             for k, v in leaves.items()})


def init_params(names_shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int = 2,
                dtype=torch.float32) -> Dict[str, torch.Tensor]:
    """Seeded uniform(-1/sqrt(fan_in), 1/sqrt(fan_in)) init (PyG Linear / torch Linear bound)."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shape in names_shapes:
        fan_in = shape[1] if len(shape) == 2 else shape[0]
        b = 1.0 / max(fan_in, 1) ** 0.5
        out[name] = ((torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1) * b).to(dtype)
    return out
