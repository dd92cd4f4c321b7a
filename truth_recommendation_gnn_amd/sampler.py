"""Neighbour-sampled mini-batches for the hetero SAGE stack (BASELINE cfg5).

The reference trains full-batch (``train_gnn.py:254``) and has no sampler.  This adds the usual
layer-wise scheme so the 4-relation 10M-node config can train on mini-batches:

* ``NeighborSampler(num_nodes, edge_index_dict, relations, fanouts)`` builds, once, the
  destination-grouped CSR of every relation on the GPU (K5, cached like the full-batch path);
* ``sample(seeds)`` walks outwards from the seed nodes: hop h keeps, for every frontier node and
  every relation into its type, all in-neighbours or ``fanouts[h]`` of them drawn uniformly without
  replacement (``hgnn_sample_neighbors``), then relabels the reached nodes into the next frontier
  (``hgnn_relabel``: previous frontier first, order kept, then new nodes in order of first
  appearance, as PyG's sampler orders them);
* each hop becomes one ``Block`` per layer: a ``RelationCSR`` per relation over local ids, so the
  layer runs on the same K1/K2 gathers and K3 projections as the full graph;
* ``forward_blocks(model, batch, x_dict)`` runs a ``HeteroSAGE`` on the blocks (differentiable).

With fanouts at least the maximum degree, the seeds' embeddings equal the full-graph forward's
(tested), which is the parity anchor for a component with no reference counterpart.
"""
from __future__ import annotations

import dataclasses
import weakref
from typing import Dict, List, Mapping, Sequence, Tuple

import torch

from . import _native as N
from . import ops
from .graph import RelationCSR, relation_csr
from .nn import HeteroSAGE, _fused_weights_layer

EdgeType = Tuple[str, str, str]


@dataclasses.dataclass
class Block:
    """One layer of a mini-batch: ``csr[et]`` maps the layer's source nodes (local ids into
    ``src_nodes``) to its destination nodes (a prefix of the source nodes of the same type)."""
    csr: Dict[EdgeType, RelationCSR]
    n_dst: Dict[str, int]
    n_src: Dict[str, int]


@dataclasses.dataclass
class MiniBatch:
    nodes: List[Dict[str, torch.Tensor]]   # nodes[0]: input nodes per type ... nodes[L]: seeds
    blocks: List[Block]                    # blocks[l]: nodes[l] -> nodes[l+1]

    def record_stream(self, stream: torch.cuda.Stream) -> None:
        """The batch was sampled on another stream and is consumed on ``stream``: keep its
        device buffers from being reused by the sampling stream until ``stream`` is done."""
        for nd in self.nodes:
            for t in nd.values():
                t.record_stream(stream)
        for blk in self.blocks:
            for c in blk.csr.values():
                c.fwd.rowptr.record_stream(stream)
                c.fwd.col.record_stream(stream)


_MAX_GROUP = 8     # relations per hop / node types per relabel / relations per CSC group


def _i32(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.int32).contiguous()


class NeighborSampler:
    def __init__(self, num_nodes: Mapping[str, int],
                 edge_index_dict: Mapping[EdgeType, torch.Tensor],
                 relations: Sequence[EdgeType], fanouts: Sequence[int]):
        if not fanouts:
            raise ValueError("fanouts: at least one hop (one per model layer)")
        if any(f == 0 or f > 64 for f in fanouts):
            raise ValueError("fanouts must be in 1..64, or < 0 for every neighbour")
        self.num_nodes = {t: int(n) for t, n in num_nodes.items()}
        self.relations = [tuple(et) for et in relations]
        self.fanouts = list(fanouts)
        # the one-launch hop kernels' limits (csrc/sampler.hip kHopMax / kRelabelMaxTypes, the
        # CSC group's kTransposeMax in csr_build.hip), checked here rather than at sample time
        types = set(self.num_nodes)
        for et in self.relations:
            if et[0] not in types or et[2] not in types:
                raise ValueError(f"relation {et}: node type without a node count")
        if len(self.relations) > _MAX_GROUP:
            raise ValueError(f"{len(self.relations)} relations: the hop kernels take at most "
                             f"{_MAX_GROUP} (one sampled block's CSCs are built by one sort)")
        if len(types) > _MAX_GROUP:
            raise ValueError(f"{len(types)} node types: the relabel takes at most {_MAX_GROUP}")
        if len(types) > 1 and max(self.num_nodes.values()) * len(types) >= 2**31 - 1:
            raise ValueError("node ids x types must stay below 2^31 (the relabel key)")
        # full-graph CSR per relation: rows = destinations, col = global source ids
        self.csr = {et: relation_csr(edge_index_dict[et], self.num_nodes[et[0]],
                                     self.num_nodes[et[2]]) for et in self.relations}
        self.device = next(iter(edge_index_dict.values())).device

    def _count(self, et: EdgeType, dst: torch.Tensor, fanout: int):
        """Phase 1 (no sync): the block rowptr of relation ``et`` for destinations ``dst``."""
        g = self.csr[et].fwd
        lib, dev = N.lib(), self.device
        n = int(dst.numel())
        rowptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
        ws = N.workspace(lib.hgnn_sample_ws_bytes(n), dev)
        N.check(lib.hgnn_sample_neighbors(N.ptr(g.rowptr), N.ptr(g.col), g.n_rows, N.ptr(dst), n,
                                          fanout, 0, N.ptr(rowptr), None, N.ptr(ws), ws.numel(),
                                          N.stream_ptr(dev)), "hgnn_sample_neighbors")
        return rowptr, ws

    def _fill(self, et: EdgeType, dst: torch.Tensor, fanout: int, seed: int, rowptr,
              total: int):
        """Phase 2 (one launch, on phase 1's rowptr): the sampled source ids (global) into a
        ``total``-long column array."""
        g = self.csr[et].fwd
        lib, dev = N.lib(), self.device
        col = torch.empty(total, dtype=torch.int32, device=dev)
        N.check(lib.hgnn_sample_fill(N.ptr(g.rowptr), N.ptr(g.col), g.n_rows, N.ptr(dst),
                                     int(dst.numel()), fanout, seed, N.ptr(rowptr), N.ptr(col),
                                     N.stream_ptr(dev)), "hgnn_sample_fill")
        return col

    def _sample(self, et: EdgeType, dst: torch.Tensor, fanout: int, seed: int):
        rowptr, _ = self._count(et, dst, fanout)
        return rowptr, self._fill(et, dst, fanout, seed, rowptr, int(rowptr[-1]))

    def _hop(self, ets, cur, fanout: int, seed: int):
        """Count + fill of every relation into the frontier in one launch per phase
        (``hgnn_sample_hop_count`` / ``_fill``) and the hop's one read-back of the sizes.  The
        kernels count ids outside the table as degree 0, so unchecked seeds are never
        dereferenced (they are checked by the first relabel).  Returns per relation its
        zero-based rowptr, the hop's column buffer (relations in ``ets`` order, adjacent) and
        the sizes."""
        lib, dev = N.lib(), self.device
        if not ets:
            return {}, torch.empty(0, dtype=torch.int32, device=dev), {}
        g = [self.csr[et].fwd for et in ets]
        dsts = [cur[et[2]] for et in ets]
        n_dst = [int(d.numel()) for d in dsts]
        n_tot = sum(n_dst)
        rp_all = torch.empty(n_tot + len(ets) + len(ets), dtype=torch.int32, device=dev)
        rps, o = [], 0
        for n in n_dst:
            rps.append(rp_all[o:o + n + 1])
            o += n + 1
        d_tot = rp_all[o:]
        ws = N.workspace(lib.hgnn_sample_hop_ws_bytes(n_tot), dev)
        R = len(ets)
        a_rp, a_dst = N.ptr_array([x.rowptr for x in g]), N.ptr_array(dsts)
        a_nr, a_nd = N.i64_array([x.n_rows for x in g]), N.i64_array(n_dst)
        a_out = N.ptr_array(rps)
        s = N.stream_ptr(dev)
        N.check(lib.hgnn_sample_hop_count(R, a_rp, a_nr, a_dst, a_nd, fanout, a_out, N.ptr(d_tot),
                                          N.ptr(ws), ws.numel(), s), "hgnn_sample_hop_count")
        totals = d_tot.tolist()                            # the hop's first sync
        # one buffer, at least one element: every relation's output address is non-null, an
        # empty relation's included (an empty tensor view reports a null data_ptr)
        buf = torch.empty(max(sum(totals), 1), dtype=torch.int32, device=dev)
        cols = buf[:sum(totals)]
        outs, o = (N._p * max(R, 1))(), 0
        for r, t in enumerate(totals):
            outs[r] = buf.data_ptr() + 4 * o
            o += t
        N.check(lib.hgnn_sample_hop_fill(R, a_rp, N.ptr_array([x.col for x in g]), a_nr, a_dst,
                                         a_nd, fanout, seed, a_out, outs, s),
                "hgnn_sample_hop_fill")
        return dict(zip(ets, rps)), cols, dict(zip(ets, totals))

    def _relabel_hop(self, types, cur, items: torch.Tensor, n_items):
        """Next node sets of every type of the hop in one call (``hgnn_relabel_multi``): type
        t's prefix is ``cur[t]`` (the previous frontier, or the seeds), its items the t-th
        consecutive range of ``items``.  Returns (nodes per type, local ids of all items,
        counts) with counts[2t] = t's node count and counts[2t+1] its prefix-check flags (read
        on the first hop, whose prefix is the seeds; later frontiers are distinct by
        construction)."""
        lib, dev = N.lib(), self.device
        empty = torch.empty(0, dtype=torch.int32, device=dev)
        prefixes = [cur.get(t, empty) for t in types]
        n_pre = [int(p.numel()) for p in prefixes]
        nodes = {t: torch.empty(max(n_pre[i] + n_items[i], 1), dtype=torch.int32, device=dev)
                 for i, t in enumerate(types)}
        local = torch.empty(max(int(items.numel()), 1), dtype=torch.int32, device=dev)
        counts = torch.zeros(2 * len(types), dtype=torch.int32, device=dev)
        ws = N.workspace(lib.hgnn_relabel_multi_ws_bytes(sum(n_pre), int(items.numel())), dev)
        items_p = N.ptr(items) if items.numel() else N.ptr(local)   # a non-null address
        N.check(lib.hgnn_relabel_multi(
            len(types), N.ptr_array(prefixes), N.i64_array(n_pre),
            N.i64_array([self.num_nodes[t] for t in types]), items_p, N.i64_array(n_items),
            N.ptr(local), N.ptr_array([nodes[t] for t in types]), N.ptr(counts), 1, N.ptr(ws),
            ws.numel(), N.stream_ptr(dev)), "hgnn_relabel_multi")
        return nodes, local[:int(items.numel())], counts

    def _relabel(self, t: str, prefix: torch.Tensor, items: torch.Tensor, check: bool = False):
        """Next node set of type ``t``; returns (nodes, local, count2): ``count2[0]`` = the
        node count, ``count2[1]`` the prefix check's flags when ``check`` (bit 0 a repeated
        prefix id, bit 1 one outside the type's id range), read back by the caller."""
        lib, dev = N.lib(), self.device
        n_p, n_i = int(prefix.numel()), int(items.numel())
        nodes = torch.empty(n_p + n_i, dtype=torch.int32, device=dev)
        local = torch.empty(n_i, dtype=torch.int32, device=dev)
        count = torch.zeros(2, dtype=torch.int32, device=dev) if check else \
            torch.empty(2, dtype=torch.int32, device=dev)
        ws = N.workspace(lib.hgnn_relabel_ws_bytes(n_p, n_i), dev)
        if check:
            N.check(lib.hgnn_relabel_checked(N.ptr(prefix), n_p, self.num_nodes[t], N.ptr(items),
                                             n_i, N.ptr(local), N.ptr(nodes), N.ptr(count),
                                             N.ptr(ws), ws.numel(), N.stream_ptr(dev)),
                    "hgnn_relabel_checked")
        else:
            N.check(lib.hgnn_relabel(N.ptr(prefix), n_p, N.ptr(items), n_i, N.ptr(local),
                                     N.ptr(nodes), N.ptr(count), N.ptr(ws), ws.numel(),
                                     N.stream_ptr(dev)), "hgnn_relabel")
        return nodes, local, count

    def sample(self, seeds: Mapping[str, torch.Tensor], seed: int = 0) -> MiniBatch:
        cur: Dict[str, torch.Tensor] = {}
        for t, s in seeds.items():
            if t not in self.num_nodes:
                raise ValueError(f"unknown node type {t!r}")
            cur[t] = _i32(s.to(self.device))
        # the seeds are checked (distinct, in range) by the first hop's relabel, whose prefix
        # they are; its flags come back with the node counts (no sync of its own)
        nodes, blocks = [cur], []
        for hop, fanout in enumerate(self.fanouts):
            hop_seed = (int(seed) * 1_000_003 + hop) & 0xFFFFFFFFFFFFFFFF
            # relations into the frontier, grouped by source type: each type's sampled items are
            # then one contiguous run of the hop's column buffer (no concatenation for relabel)
            types = sorted(set(cur) | {et[0] for et in self.relations if et[2] in cur})
            ets = sorted((et for et in self.relations if et[2] in cur),
                         key=lambda et: types.index(et[0]))
            rowptr, cols, totals = self._hop(ets, cur, fanout, hop_seed)
            n_items = [sum(totals[et] for et in ets if et[0] == t) for t in types]
            nodes_t, local_all, counts = self._relabel_hop(types, cur, cols, n_items)
            vals = counts.tolist()                                         # one sync per hop
            sizes = vals[0::2]
            if hop == 0:
                for t, flags in zip(types, vals[1::2]):
                    if flags & 2:
                        raise ValueError(f"seed ids of type {t!r} out of range")
                    if flags & 1:
                        raise ValueError(f"seed ids of type {t!r} must be distinct")
            nxt: Dict[str, torch.Tensor] = {t: nodes_t[t][:n] for t, n in zip(types, sizes)}
            local: Dict[EdgeType, torch.Tensor] = {}
            o = 0
            for et in ets:                       # ets are grouped by source type in `types` order
                local[et] = local_all[o:o + totals[et]]
                o += totals[et]
            csrs = {et: RelationCSR.from_csr(rowptr[et], local[et], int(nxt[et[0]].numel()),
                                             int(cur[et[2]].numel()),
                                             may_have_heavy_rows=fanout < 0)
                    for et in ets}
            group = [weakref.ref(c) for c in csrs.values()]   # the block's backward CSCs:
            for c in csrs.values():                           # one sort for all of them
                c._csc_group = group
            blocks.append(Block(csrs, {t: int(v.numel()) for t, v in cur.items()},
                                {t: int(v.numel()) for t, v in nxt.items()}))
            nodes.append(nxt)
            cur = nxt
        return MiniBatch(nodes[::-1], blocks[::-1])


def forward_blocks(model: HeteroSAGE, batch: MiniBatch,
                   x_dict: Mapping[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """``model`` on the sampled blocks; returns the seeds' embeddings per type (seed order)."""
    if len(batch.blocks) != len(model.layers):
        raise ValueError(f"{len(batch.blocks)} blocks for a {len(model.layers)}-layer model")
    h = {t: x_dict[t].index_select(0, ids) for t, ids in batch.nodes[0].items()}   # int32 ids
    for convs, blk in zip(model.layers, batch.blocks):
        # one fused hetero layer per block (ops.hetero_layer: per destination type the K1 means of
        # its relations and one K3 over [aggr..., root prefix], one autograd node for the layer)
        out, groups, msgs_g = {}, [], []
        for dst, n_dst in blk.n_dst.items():
            msgs = [("__".join(et), et, w) for et, w in model.relations
                    if et[2] == dst and et in blk.csr]
            if not msgs:                      # no relation into this type: kept as is
                out[dst] = h[dst][:n_dst]
                continue
            rels = tuple((et[0], blk.csr[et]) for _, et, _ in msgs)
            groups.append(ops.DstGroup(dst, rels, True, True, (), n_root=n_dst))
            msgs_g.append(msgs)
        if groups:
            out.update(ops.hetero_layer(ops.LayerSpec(tuple(sorted(h)), tuple(groups)), h,
                                        _fused_weights_layer(convs, msgs_g, h)))
        h = out
    return h
