"""Graph container and the device-resident CSR/CSC cache.

``HeteroData`` is the slice of PyG's container the reference uses (``train_gnn.py:115-142,
211-216``; ``test_gnn.py:73-109``; ``inference.py:410-419``): ``graph['user'].x = ...``,
``graph['user','social','user'].edge_index = ...``, ``graph.to(device)``,
``graph.edge_index_dict``, ``graph['user'].num_nodes``.

``RelationCSR`` is what the kernels walk: for a COO ``edge_index`` [2,E] (row 0 = source,
row 1 = destination, PyG's source_to_target flow) it holds the stable CSR grouped by destination
(forward gather, K1) and, on demand, the stable CSC grouped by source (backward, K2), 1/deg, and
the degree-skew plans.  Built on the GPU by K5 once per graph and cached, keyed by the edge
tensor's storage pointer, version counter and shape.
"""
from __future__ import annotations

import collections
import dataclasses
import weakref
from typing import Dict, Optional, Tuple

import torch

from . import _native as N

EdgeType = Tuple[str, str, str]


# ----------------------------------------------------------------------------- HeteroData (lite)
class _Storage:
    def __init__(self):
        object.__setattr__(self, "_d", {})

    def __getattr__(self, k):
        d = object.__getattribute__(self, "_d")
        if k in d:
            return d[k]
        raise AttributeError(k)

    def __setattr__(self, k, v):
        self._d[k] = v

    def __contains__(self, k):
        return k in self._d

    def items(self):
        return self._d.items()


class NodeStorage(_Storage):
    @property
    def num_nodes(self) -> int:
        return int(self._d["x"].shape[0])


class EdgeStorage(_Storage):
    @property
    def num_edges(self) -> int:
        return int(self._d["edge_index"].shape[1])


class HeteroData:
    """Minimal PyG ``HeteroData``: node stores keyed by type, edge stores by (src, rel, dst)."""

    def __init__(self):
        self._nodes: Dict[str, NodeStorage] = {}
        self._edges: Dict[EdgeType, EdgeStorage] = {}

    def __getitem__(self, key):
        if isinstance(key, str):
            return self._nodes.setdefault(key, NodeStorage())
        if isinstance(key, tuple) and len(key) == 3:
            return self._edges.setdefault(tuple(key), EdgeStorage())
        raise KeyError(key)

    @property
    def node_types(self):
        return list(self._nodes)

    @property
    def edge_types(self):
        return list(self._edges)

    def metadata(self):
        return self.node_types, self.edge_types

    @property
    def x_dict(self) -> Dict[str, torch.Tensor]:
        return {k: v.x for k, v in self._nodes.items() if "x" in v}

    @property
    def edge_index_dict(self) -> Dict[EdgeType, torch.Tensor]:
        return {k: v.edge_index for k, v in self._edges.items() if "edge_index" in v}

    def to(self, device) -> "HeteroData":
        for store in list(self._nodes.values()) + list(self._edges.values()):
            for k, v in list(store.items()):
                if torch.is_tensor(v):
                    setattr(store, k, v.to(device))
        return self


# ----------------------------------------------------------------------------- CSR cache
def default_chunk(num_edges: int) -> int:
    """Split rows longer than about a quarter of one wave's share of the edges
    (cdna_hip_programming.md App. B 'Scatter / gather'): 256 CUs x 32 waves in flight."""
    share = max(num_edges // (256 * 32 * 4), 1)
    c = 1 << (share.bit_length() - 1)
    return int(min(max(c, 64), 1024))


# chunk of a plan without heavy rows when the rows were not counted: no row is ever split (the
# gather kernels skip a row longer than the chunk in its light pass, leaving it to the heavy list)
NO_SPLIT = 1 << 30


@dataclasses.dataclass
class Plan:
    chunk: int
    n_heavy: int
    n_chunks: int
    heavy_rows: Optional[torch.Tensor]
    heavy_first: Optional[torch.Tensor]


@dataclasses.dataclass
class GroupedEdges:
    rowptr: torch.Tensor     # int32 [n_rows+1]
    col: torch.Tensor        # int32 [E]
    perm: Optional[torch.Tensor]   # int32 [E] original edge id of each CSR position (None: the
    #                                identity, for edges that came grouped — RelationCSR.from_csr)
    plan: Plan
    n_rows: int


def _plan(rowptr: torch.Tensor, n_rows: int, chunk: int) -> Plan:
    dev = rowptr.device
    if n_rows == 0:
        return Plan(chunk, 0, 0, None, None)
    lib, s = N.lib(), N.stream_ptr(dev)
    ws = N.workspace(lib.hgnn_plan_ws_bytes(n_rows), dev)
    counts = torch.zeros(2, dtype=torch.int32, device=dev)
    N.check(lib.hgnn_plan_count(N.ptr(rowptr), n_rows, chunk, N.ptr(counts), N.ptr(ws),
                                ws.numel(), s), "hgnn_plan_count")
    n_heavy, n_chunks = (int(v) for v in counts.tolist())   # host sync: once per graph
    if n_heavy == 0:
        return Plan(chunk, 0, 0, None, None)
    heavy_rows = torch.empty(n_heavy, dtype=torch.int32, device=dev)
    heavy_first = torch.empty(n_heavy + 1, dtype=torch.int32, device=dev)
    N.check(lib.hgnn_plan_fill(N.ptr(rowptr), n_rows, chunk, N.ptr(heavy_rows),
                               N.ptr(heavy_first), N.ptr(ws), ws.numel(), s), "hgnn_plan_fill")
    return Plan(chunk, n_heavy, n_chunks, heavy_rows, heavy_first)


def group_edges(key: torch.Tensor, other: torch.Tensor, n_keys: int, n_other: int,
                chunk: Optional[int] = None) -> GroupedEdges:
    """K5: stable grouping of COO by ``key`` (int64 device tensors) -> CSR + skew plan."""
    dev = N.require_device(key, other)
    E = int(key.numel())
    if E >= 2**31 - 1 or n_keys >= 2**31 - 1 or n_other >= 2**31 - 1:
        raise ValueError(f"graph too large for int32 CSR: E={E} n_keys={n_keys}")
    key = key.contiguous().to(torch.int64)
    other = other.contiguous().to(torch.int64)
    lib, s = N.lib(), N.stream_ptr(dev)
    rowptr = torch.empty(n_keys + 1, dtype=torch.int32, device=dev)
    col = torch.empty(E, dtype=torch.int32, device=dev)
    perm = torch.empty(E, dtype=torch.int32, device=dev)
    invalid = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = N.workspace(lib.hgnn_coo_to_csr_ws_bytes(E, n_keys), dev)
    N.check(lib.hgnn_coo_to_csr(N.ptr(key), N.ptr(other), E, n_keys, n_other, N.ptr(rowptr),
                                N.ptr(col), N.ptr(perm), N.ptr(invalid), N.ptr(ws), ws.numel(), s),
            "hgnn_coo_to_csr")
    bad = int(invalid.item())   # host sync: once per graph
    if bad:
        raise ValueError(f"edge_index has {bad} edge(s) with an endpoint out of range "
                         f"(n_keys={n_keys}, n_other={n_other}); the reference masks these out "
                         "before building the graph (train_gnn.py:128-133)")
    c = chunk if chunk is not None else default_chunk(E)
    return GroupedEdges(rowptr, col, perm, _plan(rowptr, n_keys, c), n_keys)


class RelationCSR:
    """Cached device structures for one relation (edge_index [2,E], n_src, n_dst)."""

    def __init__(self, edge_index: torch.Tensor, n_src: int, n_dst: int,
                 chunk: Optional[int] = None):
        if edge_index.dim() != 2 or edge_index.shape[0] != 2:
            raise ValueError(f"edge_index must be [2, E], got {tuple(edge_index.shape)}")
        self.n_src, self.n_dst = int(n_src), int(n_dst)
        self.num_edges = int(edge_index.shape[1])
        self.chunk = chunk
        # the COO is held weakly: the CSR cache keys on the edge tensor's lifetime, and a strong
        # reference here would keep every cached tensor (and so its entry) alive.  When the tensor
        # is gone (or changed in place) the COO is rebuilt from the CSR (see edge_index).
        self._ei = None
        self._ei_ref = weakref.ref(edge_index)
        self._ei_version = edge_index._version
        self.fwd = group_edges(edge_index[1], edge_index[0], self.n_dst, self.n_src, chunk)
        self._inv_deg: Optional[torch.Tensor] = None
        self._bwd: Optional[GroupedEdges] = None

    @property
    def inv_deg(self) -> torch.Tensor:
        """1/deg per destination row (0 for an empty row), on first use."""
        if self._inv_deg is None:
            dev = self.fwd.rowptr.device
            self._inv_deg = torch.empty(self.n_dst, dtype=torch.float32, device=dev)
            N.check(N.lib().hgnn_inv_degree(N.ptr(self.fwd.rowptr), self.n_dst,
                                            N.ptr(self._inv_deg), N.stream_ptr(dev)),
                    "hgnn_inv_degree")
        return self._inv_deg

    @classmethod
    def from_csr(cls, rowptr: torch.Tensor, col: torch.Tensor, n_src: int, n_dst: int,
                 may_have_heavy_rows: bool = True) -> "RelationCSR":
        """A relation whose edges already come grouped by destination (``rowptr`` over n_dst
        rows, ``col`` = source ids): no sort and no validation sync.  The edge ids are the CSR
        positions; the COO and the transposed grouping are derived on first use.  Rows are
        short (e.g. sampled blocks) unless ``may_have_heavy_rows``, which builds the skew plan."""
        self = cls.__new__(cls)
        self.n_src, self.n_dst = int(n_src), int(n_dst)
        self.num_edges = int(col.numel())
        self.chunk = None
        c = default_chunk(self.num_edges)
        plan = (_plan(rowptr, self.n_dst, c) if may_have_heavy_rows
                else Plan(NO_SPLIT, 0, 0, None, None))
        # nothing else is launched here: a sampled mini-batch builds eight of these per step, and
        # 1/deg and the CSC are needed only by the backward (layers whose input has a gradient)
        self.fwd = GroupedEdges(rowptr, col, None, plan, self.n_dst)
        self._inv_deg = None
        self._ei = None
        self._bwd = None
        self._from_csr = True
        return self

    def _dst_of_positions(self, dtype) -> torch.Tensor:
        g = self.fwd
        deg = g.rowptr[1:] - g.rowptr[:-1]
        return torch.repeat_interleave(torch.arange(self.n_dst, dtype=dtype, device=g.col.device),
                                       deg, output_size=self.num_edges)   # no host sync

    @property
    def edge_index(self) -> torch.Tensor:
        """[2, E] COO (source, destination): the caller's tensor while it lives unchanged;
        otherwise rebuilt from the CSR — in the original edge order (``fwd.perm`` holds each CSR
        position's COO id), or in CSR order for a relation built ``from_csr``."""
        if self._ei is not None:
            return self._ei
        ref = getattr(self, "_ei_ref", None)
        t = ref() if ref is not None else None
        if t is not None and t._version == self._ei_version:
            return t
        g = self.fwd
        coo = torch.stack([g.col.long(), self._dst_of_positions(torch.int64)])
        if g.perm is None:
            self._ei = coo            # from_csr: CSR order is the relation's edge order
            return coo
        out = torch.empty_like(coo)
        out[:, g.perm.long()] = coo
        return out                    # not kept: needed once per structure built from it

    @property
    def bwd(self) -> GroupedEdges:
        """Transposed grouping (by source), built on first backward that needs it."""
        if self._bwd is None:
            if getattr(self, "_from_csr", False):
                self._bwd = self._bwd_from_csr()
            else:
                ei = self.edge_index
                self._bwd = group_edges(ei[0], ei[1], self.n_src, self.n_dst, self.chunk)
        return self._bwd

    def _bwd_from_csr(self) -> GroupedEdges:
        """CSC of a relation built ``from_csr`` (sampled blocks), in one call
        (``hgnn_csr_transpose``): the ids were produced on the device and are valid by
        construction, so there is no validation pass and no host sync, and the same call writes
        the per-position 1/deg that K2 streams (``bwd_weights``).  No skew plan (it needs a host
        sync to size): a source row is summed by one wave however long it is — a hot post drawn
        by many sampled edges included (at cfg5, 700+ of one block's 15k rev_engages edges)."""
        group = getattr(self, "_csc_group", None)     # weak references to the block's relations
        if group is not None:
            members = [m for m in (ref() for ref in group) if m is not None]
            if any(m is self for m in members):
                build_csc_group(members)     # every relation of the block in one sort
                return self._bwd
        g, E = self.fwd, self.num_edges
        dev = g.col.device
        rowptr = torch.empty(self.n_src + 1, dtype=torch.int32, device=dev)
        col = torch.empty(E, dtype=torch.int32, device=dev)
        perm = torch.empty(E, dtype=torch.int32, device=dev)
        w = torch.empty(E, dtype=torch.float32, device=dev)
        lib = N.lib()
        ws = N.workspace(lib.hgnn_sort_pairs_ws_bytes(E, self.n_src), dev)
        N.check(lib.hgnn_csr_transpose(N.ptr(g.rowptr), N.ptr(g.col), self.n_dst, E, self.n_src,
                                       N.ptr(rowptr), N.ptr(col), N.ptr(perm), N.ptr(w),
                                       N.ptr(ws), ws.numel(), N.stream_ptr(dev)),
                "hgnn_csr_transpose")
        self._bwd_w = w
        return GroupedEdges(rowptr, col, perm, Plan(NO_SPLIT, 0, 0, None, None), self.n_src)

    @property
    def bwd_weights(self) -> torch.Tensor:
        """1/deg(dst) per CSC position (static): K2 streams it instead of a dependent random
        lookup of inv_deg[dst] per edge."""
        w = getattr(self, "_bwd_w", None)
        if w is None:
            g = self.bwd                  # (a from_csr relation's CSC build sets _bwd_w too)
            w = getattr(self, "_bwd_w", None)
        if w is None:
            w = self.inv_deg[g.col.long()].contiguous() if self.num_edges else \
                torch.empty(0, dtype=torch.float32, device=self.inv_deg.device)
            self._bwd_w = w
        return w

    def blocks(self, side: str, n_blocks: int):
        """The relation split into ``n_blocks`` passes over contiguous blocks of the table a
        gather reads: ``side="fwd"`` (K1, reads the sources; rows = destinations) blocks by
        source id, ``side="bwd"`` (K2, reads the destinations' gradients; rows = sources) by
        destination id.  Returns (passes, weights): one GroupedEdges per block (its rowptr a slice
        of one CSR keyed by (block, row) — absolute offsets into a shared col — with its own skew
        plan), and for "bwd" the 1/deg(destination) per position in that order.  Built once (one
        K5 sort) and cached; see ops.GATHER_BLOCK_BYTES for why."""
        key = (side, int(n_blocks))
        cache = self.__dict__.setdefault("_blocks", {})
        if key in cache:
            return cache[key]
        B = int(n_blocks)
        n_rows_side = self.n_dst if side == "fwd" else self.n_src
        if B * n_rows_side >= 2**31 - 1:
            raise ValueError(f"blocks: {B} passes x {n_rows_side} rows exceed the int32 rowptr")
        ei = self.edge_index
        if side == "fwd":
            n_rows, n_read, rows, reads = self.n_dst, self.n_src, ei[1], ei[0]
        else:
            n_rows, n_read, rows, reads = self.n_src, self.n_dst, ei[0], ei[1]
        bs = -(-n_read // B)
        ge = group_edges((reads // bs) * n_rows + rows, reads, B * n_rows, n_read, chunk=NO_SPLIT)
        chunk = default_chunk(max(self.num_edges // B, 1))
        passes = []
        for b in range(B):
            rp = ge.rowptr[b * n_rows:(b + 1) * n_rows + 1]
            passes.append(GroupedEdges(rp, ge.col, None, _plan(rp, n_rows, chunk), n_rows))
        w = self.inv_deg[ge.col.long()].contiguous() if side == "bwd" else None
        cache[key] = (passes, w)
        return cache[key]

    def release_coo(self):
        """Drop the COO reference once the CSC exists (saves 16 B/edge of HBM)."""
        if self._bwd is not None:
            self._ei = None


def build_csc_group(rels) -> None:
    """The CSCs (and K2 weights) of several ``RelationCSR.from_csr`` relations — one sampled
    block's — in one sort (``hgnn_csr_transpose_multi``), cached on each relation.  A block's
    backward needs all of them, so the first relation asked builds the group."""
    rels = [r for r in rels if r._bwd is None]
    if not rels:
        return
    dev = rels[0].fwd.col.device
    outs = []
    for r in rels:
        E = r.num_edges
        outs.append((torch.empty(r.n_src + 1, dtype=torch.int32, device=dev),
                     torch.empty(max(E, 1), dtype=torch.int32, device=dev),
                     torch.empty(max(E, 1), dtype=torch.int32, device=dev),
                     torch.empty(max(E, 1), dtype=torch.float32, device=dev)))
    lib = N.lib()
    Es = [r.num_edges for r in rels]
    ws = N.workspace(lib.hgnn_csr_transpose_multi_ws_bytes(sum(Es), sum(r.n_src for r in rels)),
                     dev)
    N.check(lib.hgnn_csr_transpose_multi(
        len(rels), N.ptr_array([r.fwd.rowptr for r in rels]),
        N.ptr_array([r.fwd.col if r.num_edges else o[1] for r, o in zip(rels, outs)]),
        N.i64_array([r.n_dst for r in rels]), N.i64_array(Es),
        N.i64_array([r.n_src for r in rels]), N.ptr_array([o[0] for o in outs]),
        N.ptr_array([o[1] for o in outs]), N.ptr_array([o[2] for o in outs]),
        N.ptr_array([o[3] for o in outs]), N.ptr(ws), ws.numel(), N.stream_ptr(dev)),
        "hgnn_csr_transpose_multi")
    for r, (rp, col, perm, w) in zip(rels, outs):
        E = r.num_edges
        r._bwd = GroupedEdges(rp, col[:E], perm[:E], Plan(NO_SPLIT, 0, 0, None, None), r.n_src)
        r._bwd_w = w[:E]


class _CsrCache:
    """Edge tensor -> its RelationCSR.  An entry lives as long as its edge tensor: a
    ``weakref.finalize`` on the tensor drops it when the tensor is freed (a caller that builds a
    fresh edge tensor per call — ``inference.py:410-419`` builds a graph per user, a per-step
    ``flip(0)`` — pins nothing), and an in-place change of the tensor (new version) replaces its
    entry.  ``cap`` bounds the entries of live tensors (least recently used dropped first)."""

    def __init__(self, cap: int = 64):
        self.cap = cap
        self._d: "collections.OrderedDict" = collections.OrderedDict()

    def __len__(self):
        return len(self._d)

    def _drop(self, key, csr_id):
        hit = self._d.get(key)
        if hit is not None and id(hit[1]) == csr_id:
            del self._d[key]

    def get(self, edge_index: torch.Tensor, n_src: int, n_dst: int,
            chunk: Optional[int] = None) -> RelationCSR:
        key = (edge_index.data_ptr(), edge_index._version, tuple(edge_index.shape),
               tuple(edge_index.stride()), edge_index.device, int(n_src), int(n_dst), chunk)
        hit = self._d.get(key)
        if hit is not None:
            ref, csr = hit
            if ref() is edge_index:
                self._d.move_to_end(key)
                return csr
        # entries of this same tensor at an older version (changed in place since) are stale
        for k in [k for k, (ref, _) in self._d.items() if ref() is edge_index]:
            del self._d[k]
        csr = RelationCSR(edge_index, n_src, n_dst, chunk)
        self._d[key] = (weakref.ref(edge_index), csr)
        weakref.finalize(edge_index, self._drop, key, id(csr))
        while len(self._d) > self.cap:
            self._d.popitem(last=False)
        return csr

    def clear(self):
        self._d.clear()


CSR_CACHE = _CsrCache()


def relation_csr(edge_index: torch.Tensor, n_src: int, n_dst: int,
                 chunk: Optional[int] = None) -> RelationCSR:
    return CSR_CACHE.get(edge_index, n_src, n_dst, chunk)
