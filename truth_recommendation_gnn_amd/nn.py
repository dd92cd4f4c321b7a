"""PyG-compatible modules over the fused HIP path.

* ``SAGEConv(in_channels, out_channels)`` — the operator the reference builds three of
  (``train_gnn.py:158-160``): ``lin_l`` (with bias) on the mean aggregate, ``lin_r`` (no bias) on
  the destination features, lazy ``(-1, -1)`` in-channels, same state_dict keys as PyG
  (``lin_l.weight``, ``lin_l.bias``, ``lin_r.weight``).
* ``WeightedRGCN(hidden_dim)`` — ``train_gnn.py:147-200`` (and ``inference.py:119-169``), same
  module names and fixed relation weights, so ``best_rgcn_model.pt`` state_dicts load unchanged;
  ``WeightedRGCNAuthor`` is the 3-message variant of ``test_gnn.py:116-168``.
* ``HeteroSAGE`` — the same relation-weighted layer stacked L times (BASELINE configs 2-5).

Every forward runs the fused per-layer op ``ops.hetero_layer`` (K1 gathers + one K3 MFMA linear
per destination type); nothing runs on the CPU.
"""
from __future__ import annotations

from typing import Dict, List, Mapping, Optional, Sequence, Tuple, Union

import torch
from torch.nn.parameter import UninitializedParameter

from . import ops
from .graph import relation_csr

EdgeType = Tuple[str, str, str]


def _linear(in_channels: int, out_channels: int, bias: bool) -> torch.nn.Module:
    """PyG ``Linear``: ``in_channels=-1`` is lazy.  Init bound 1/sqrt(fan_in) for weight and bias
    (PyG kaiming_uniform(a=sqrt(5)) == torch.nn.Linear's default)."""
    if in_channels is None or in_channels < 0:
        return torch.nn.LazyLinear(out_channels, bias=bias)
    return torch.nn.Linear(in_channels, out_channels, bias=bias)


def _materialize(lin: torch.nn.Module, in_features: int) -> None:
    if isinstance(lin, torch.nn.LazyLinear) and isinstance(lin.weight, UninitializedParameter):
        dev = lin.weight.device
        lin.initialize_parameters(torch.empty(0, in_features, device=dev))
    if isinstance(lin, torch.nn.LazyLinear) and not lin.has_uninitialized_params():
        # materialised by load_state_dict (its load hook does not set in_features)
        lin.in_features = int(lin.weight.shape[1])
        # what LazyModuleMixin._infer_parameters does after the first call
        lin._initialize_hook.remove()
        lin._load_hook.remove()
        delattr(lin, "_initialize_hook")
        delattr(lin, "_load_hook")
        lin.__class__ = torch.nn.Linear
    if lin.in_features != in_features:
        raise ValueError(f"linear expects {lin.in_features} input features, got {in_features}")


class SAGEConv(torch.nn.Module):
    """GraphSAGE operator with PyG's defaults: mean aggregation over ``edge_index`` (row 0 =
    source, row 1 = destination), ``out = lin_l(aggr) + lin_r(x_dst)``."""

    def __init__(self, in_channels: Union[int, Tuple[int, int]], out_channels: int,
                 aggr: str = "mean", normalize: bool = False, root_weight: bool = True,
                 project: bool = False, bias: bool = True):
        super().__init__()
        if aggr != "mean" or normalize or project:
            raise NotImplementedError("hgnn implements SAGEConv(aggr='mean', normalize=False, "
                                      "project=False) — the configuration the reference uses")
        if isinstance(in_channels, int):
            in_channels = (in_channels, in_channels)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.root_weight = root_weight
        self.lin_l = _linear(in_channels[0], out_channels, bias)
        self.lin_r = _linear(in_channels[1], out_channels, False) if root_weight else None

    def reset_parameters(self):
        for lin in (self.lin_l, self.lin_r):
            if lin is not None and not isinstance(lin.weight, UninitializedParameter):
                lin.reset_parameters()

    def materialize(self, d_src: int, d_dst: Optional[int]) -> None:
        _materialize(self.lin_l, d_src)
        if self.lin_r is not None and d_dst is not None:
            _materialize(self.lin_r, d_dst)

    def forward(self, x, edge_index: torch.Tensor, size=None) -> torch.Tensor:
        if torch.is_tensor(x):
            x = (x, x)
        x_src, x_dst = x
        n_dst = x_dst.shape[0] if x_dst is not None else (size[1] if size else x_src.shape[0])
        root = self.root_weight and x_dst is not None
        self.materialize(x_src.shape[1], x_dst.shape[1] if root else None)
        csr = relation_csr(edge_index, x_src.shape[0], n_dst)
        if root:
            w = torch.cat([self.lin_l.weight, self.lin_r.weight], dim=1)
            xd = {"src": x_src, "dst": x_dst}
        else:
            w = self.lin_l.weight
            xd = {"src": x_src, "dst": x_src.new_empty(n_dst, 0)}
        spec = ops.LayerSpec(("src", "dst"), (ops.DstGroup("dst", (("src", csr),), root, False),))
        return ops.hetero_layer(spec, xd, [(w, self.lin_l.bias)])["dst"]

    def __repr__(self):
        return f"{type(self).__name__}({self.in_channels}, {self.out_channels}, aggr=mean)"


# Relation layout: destination type -> [(conv name, edge type, fixed weight)]
Layout = Dict[str, List[Tuple[str, EdgeType, float]]]


def _fused_weights(convs: Dict[str, SAGEConv], msgs, x_dict) -> Tuple[torch.Tensor,
                                                                        Optional[torch.Tensor]]:
    """[w_1 W_l,1 | ... | w_R W_l,R | sum_r w_r W_r,r] and sum_r w_r b_r (autograd-tracked),
    built by one HIP launch from the per-conv parameters (``ops.fuse_weights``)."""
    wl, wr, bl, scales = [], [], [], []
    for name, et, wt in msgs:
        conv = convs[name]
        conv.materialize(x_dict[et[0]].shape[1], x_dict[et[2]].shape[1])
        wl.append(conv.lin_l.weight)
        wr.append(conv.lin_r.weight if conv.lin_r is not None else None)
        bl.append(conv.lin_l.bias)
        scales.append(wt)
    return ops.fuse_weights(wl, wr, bl, scales)


def _weight_group(convs: Dict[str, SAGEConv], msgs, dims: Mapping[str, int]):
    wl, wr, bl, scales = [], [], [], []
    for name, et, wt in msgs:
        conv = convs[name]
        conv.materialize(dims[et[0]], dims[et[2]])
        wl.append(conv.lin_l.weight)
        wr.append(conv.lin_r.weight if conv.lin_r is not None else None)
        bl.append(conv.lin_l.bias)
        scales.append(wt)
    return wl, wr, bl, scales


def _fused_weights_layer(convs: Dict[str, SAGEConv], msgs_per_group, x_dict
                         ) -> List[Tuple[torch.Tensor, Optional[torch.Tensor]]]:
    """``_fused_weights`` of every destination update of a layer, in one launch each way
    (``ops.fuse_weights_multi``)."""
    dims = {t: int(x.shape[1]) for t, x in x_dict.items()}
    return ops.fuse_weights_multi([_weight_group(convs, m, dims) for m in msgs_per_group])


def _fused_weights_layers(layers) -> List[List[Tuple[torch.Tensor, Optional[torch.Tensor]]]]:
    """``_fused_weights_layer`` of several layers — ``layers``: (convs, msgs per group, input
    width per type) each — in one launch each way when they hold at most 4 updates in all (a
    2-layer sampled step: its fuse and its split are one graph node each)."""
    groups = [[_weight_group(convs, m, dims) for m in msgs_g] for convs, msgs_g, dims in layers]
    flat = [g for gs in groups for g in gs]
    if len(flat) > 4:
        return [ops.fuse_weights_multi(gs) for gs in groups]
    out, it = [], iter(ops.fuse_weights_multi(flat))
    for gs in groups:
        out.append([next(it) for _ in gs])
    return out


class _LayoutModel(torch.nn.Module):
    """A hetero SAGE layer described by a layout, run as one fused ``hetero_layer``."""
    layout: Layout

    def _run_layer(self, convs, x_dict, edge_index_dict, relu: bool = True):
        types = tuple(sorted(x_dict))
        groups = []
        for dst, msgs in self.layout.items():
            rels = []
            for name, et, _ in msgs:
                ei = edge_index_dict[et]
                rels.append((et[0], relation_csr(ei, x_dict[et[0]].shape[0],
                                                 x_dict[dst].shape[0])))
            root = any(convs[name].lin_r is not None for name, _, _ in msgs)
            groups.append(ops.DstGroup(dst, tuple(rels), root, relu))
        weights = _fused_weights_layer(convs, list(self.layout.values()), x_dict)
        return ops.hetero_layer(ops.LayerSpec(types, tuple(groups)), dict(x_dict), weights)


class WeightedRGCN(_LayoutModel):
    """``train_gnn.py:147-200``: user = relu(1.0*msg_direct + 0.75*msg_social), post =
    relu(post_update)."""

    def __init__(self, hidden_dim: int = 64):
        super().__init__()
        self.msg_direct = SAGEConv((-1, -1), hidden_dim)
        self.msg_social = SAGEConv((-1, -1), hidden_dim)
        self.post_update = SAGEConv((-1, -1), hidden_dim)
        self.w_direct = 1.0
        self.w_social = 0.75

    @property
    def layout(self) -> Layout:
        return {
            "user": [("msg_direct", ("post", "rev_engages", "user"), self.w_direct),
                     ("msg_social", ("user", "social", "user"), self.w_social)],
            "post": [("post_update", ("user", "engages", "post"), 1.0)],
        }

    def forward(self, x_dict, edge_index_dict):
        convs = {"msg_direct": self.msg_direct, "msg_social": self.msg_social,
                 "post_update": self.post_update}
        return self._run_layer(convs, x_dict, edge_index_dict)


class WeightedRGCNAuthor(_LayoutModel):
    """``test_gnn.py:116-168``: 3 user messages weighted 1.75 / 0.7 / 0.3."""

    def __init__(self, hidden_dim: int = 64):
        super().__init__()
        self.msg_direct = SAGEConv((-1, -1), hidden_dim)
        self.msg_author = SAGEConv((-1, -1), hidden_dim)
        self.msg_social = SAGEConv((-1, -1), hidden_dim)
        self.post_update = SAGEConv((-1, -1), hidden_dim)
        self.w_direct, self.w_author, self.w_social = 1.75, 0.7, 0.3

    @property
    def layout(self) -> Layout:
        return {
            "user": [("msg_direct", ("post", "rev_engages", "user"), self.w_direct),
                     ("msg_author", ("post", "followed_by", "user"), self.w_author),
                     ("msg_social", ("user", "social", "user"), self.w_social)],
            "post": [("post_update", ("user", "engages", "post"), 1.0)],
        }

    def forward(self, x_dict, edge_index_dict):
        convs = {n: getattr(self, n) for n in ("msg_direct", "msg_author", "msg_social",
                                               "post_update")}
        return self._run_layer(convs, x_dict, edge_index_dict)


class HeteroSAGE(torch.nn.Module):
    """``num_layers`` relation-weighted SAGE layers, ReLU after each (the reference layer,
    stacked).  ``relations``: [(edge_type, weight)].  Parameters are named
    ``layers.{l}.{src}__{rel}__{dst}.lin_{l,r}.*``."""

    def __init__(self, hidden_dim: int, relations: Sequence[Tuple[EdgeType, float]],
                 num_layers: int = 2, in_channels: int = -1):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.relations = [(tuple(et), float(w)) for et, w in relations]
        self.layers = torch.nn.ModuleList()
        for l in range(num_layers):
            cin = in_channels if l == 0 else hidden_dim
            self.layers.append(torch.nn.ModuleDict(
                {"__".join(et): SAGEConv((cin, cin), hidden_dim) for et, _ in self.relations}))

    def forward(self, x_dict, edge_index_dict):
        h = dict(x_dict)
        dsts = sorted({et[2] for et, _ in self.relations})
        for convs in self.layers:
            types = tuple(sorted(h))
            groups, msgs_g = [], []
            for dst in dsts:
                msgs = [("__".join(et), et, w) for et, w in self.relations if et[2] == dst]
                rels = tuple((et[0], relation_csr(edge_index_dict[et], h[et[0]].shape[0],
                                                  h[dst].shape[0])) for _, et, _ in msgs)
                pre = tuple(ops.use_pre_projection(h[et[0]], h[dst], self.hidden_dim, True)
                            for _, et, _ in msgs)
                groups.append(ops.DstGroup(dst, rels, True, True, pre))
                msgs_g.append(msgs)
            weights = _fused_weights_layer(convs, msgs_g, h)
            out = ops.hetero_layer(ops.LayerSpec(types, tuple(groups)), h, weights)
            for t in h:
                out.setdefault(t, h[t])
            h = out
        return h
