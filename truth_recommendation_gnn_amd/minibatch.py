"""A neighbour-sampled mini-batch step replayed as one HIP graph (BASELINE cfg5).

``sampler.forward_blocks`` issues ~120 launches per step from Python and the autograd engine: at
cfg5 the step is bound by host issue (2.1 ms of host work per step against ~1.2 ms of GPU work,
``scripts/cfg5_breakdown.py``).  A graph needs fixed shapes, and every sampled batch has its own
node and edge counts, so this module runs the model on STATIC-CAPACITY blocks:

* capacities follow from the seeds and fanouts alone: level 0 holds the seeds, level h + 1 at
  most level h plus fanout x level-h destinations per relation out of each source type; every
  level gets ``slack`` padded rows on top (>= 1 padded destination row for the padding edges,
  and a padded source row for them to read);
* ``load(batch)`` copies the batch's block CSRs into the fixed buffers in ONE launch
  (``hgnn_pad_csr_multi``): real rows first and unchanged, the padding entries spread over the
  padded rows and pointing at a padded source row, so every buffer is a valid CSR of exactly its
  capacity; the outermost block's column ids are mapped to GLOBAL ids on the way, so its
  gathers read the feature tables directly (no ``index_select`` of the input nodes), and its
  destinations' own rows come as a separate root input (``DstGroup.root_src``);
* ``capture(loss_fn, optimizer)`` records forward + loss + backward (+ the optimizer step) once;
  ``step(batch)`` = ``load`` + ``replay``.

Padded rows carry finite junk (means of padded source rows) that never reaches a seed: a padded
destination row is never a source of a real row, and the loss reads the seed rows only, so the
padded rows' gradients are exactly 0 and add nothing to the weight gradients.  The block CSCs
and 1/deg the backward needs are built INSIDE the graph (the relation objects used for capture
are fresh, so nothing cached from the warm-up stands in for the next batch's structures).
Tested against the eager ``forward_blocks`` step on the same batches (outputs, loss, every
parameter gradient).
"""
from __future__ import annotations

import dataclasses
import weakref
from typing import Callable, Dict, List, Mapping, Optional, Tuple

import torch

from . import _native as N
from . import ops
from .graph import RelationCSR
from .nn import HeteroSAGE, _fused_weights
from .sampler import EdgeType, MiniBatch, NeighborSampler

SLACK = 1024


def capacities(relations, n_seeds: Mapping[str, int], fanouts, slack: int = SLACK):
    """(node capacity per level and type, edge capacity per hop and relation).  Level 0 = the
    seeds; hop h samples into level h from level h + 1 (as ``NeighborSampler.sample``: the
    relations into the level's types, the frontier first, then every sampled source)."""
    if any(f <= 0 for f in fanouts):
        raise ValueError("static blocks need bounded fanouts (every fanout > 0)")
    real = [dict(n_seeds)]
    ecap: List[Dict[EdgeType, int]] = []
    for f in fanouts:
        cur = real[-1]
        ets = [tuple(et) for et in relations if et[2] in cur]
        nxt = dict(cur)
        e = {}
        for et in ets:
            e[et] = cur[et[2]] * f
            nxt[et[0]] = nxt.get(et[0], 0) + e[et]
        ecap.append(e)
        real.append(nxt)
    cap = [{t: n + slack for t, n in lvl.items()} for lvl in real]
    return cap, ecap


class StaticBlocks:
    """Fixed-capacity buffers for the blocks of one sampler configuration (see module doc).

    ``partial_seeds``: a batch may hold FEWER seeds than ``n_seeds`` (the rest are padded level-0
    rows).  Only a loss that reads the seed rows by their local ids may allow it (``LinkLoss``:
    a link batch's distinct endpoints vary in number); a loss over all seed rows would be fed
    the padding, so by default a batch must have exactly ``n_seeds`` seeds per type."""

    def __init__(self, smp: NeighborSampler, n_seeds: Mapping[str, int], slack: int = SLACK,
                 partial_seeds: bool = False):
        self.smp = smp
        self.n_seeds = {t: int(n) for t, n in n_seeds.items()}
        self.partial_seeds = bool(partial_seeds)
        if slack < 1:
            raise ValueError("slack: at least one padded row per level")
        self.slack = int(slack)
        self.L = len(smp.fanouts)
        self.cap, self.ecap = capacities(smp.relations, self.n_seeds, smp.fanouts, slack)
        if max(max(c.values()) for c in self.cap) >= 2**31 - 1:
            raise ValueError("static block capacities exceed int32")
        dev = smp.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.rowptr = [{et: torch.empty(self.cap[h][et[2]] + 1, **i32) for et in self.ecap[h]}
                       for h in range(self.L)]
        self.col = [{et: torch.empty(max(self.ecap[h][et], 1), **i32) for et in self.ecap[h]}
                    for h in range(self.L)]
        # the outermost block's destinations (level L - 1) as global ids: its root rows
        self.root_ids = {t: torch.zeros(n, **i32) for t, n in self.cap[self.L - 1].items()}
        self.csrs: Optional[List[Dict[EdgeType, RelationCSR]]] = None

    # -- per batch ---------------------------------------------------------------------------
    def load(self, mb: MiniBatch) -> None:
        """The batch's blocks into the fixed buffers: one launch, no sync."""
        if len(mb.blocks) != self.L:
            raise ValueError(f"{len(mb.blocks)} blocks for {self.L} static levels")
        seeds = mb.nodes[-1]
        got = {t: int(v.numel()) for t, v in seeds.items()}
        if set(got) != set(self.n_seeds) or any(got[t] > self.n_seeds[t] for t in got):
            raise ValueError(f"batch seeds {got} exceed the captured capacity {self.n_seeds}")
        if not self.partial_seeds and got != self.n_seeds:
            # fewer seeds than the capacity leave padded level-0 rows, which a loss over all
            # the seed rows would read: allowed only with partial_seeds (see the class doc)
            raise ValueError(f"batch seeds {got} differ from the captured {self.n_seeds} "
                             "(partial_seeds=False)")
        L = self.L
        rp, col, mp, nd, e, rpo, colo, dcap, ecap, dummy, spread = ([] for _ in range(11))
        for h in range(L):
            blk = mb.blocks[L - 1 - h]
            if set(blk.csr) != set(self.ecap[h]):
                raise ValueError(f"hop {h}: relations {sorted(blk.csr)} differ from the static "
                                 f"layout {sorted(self.ecap[h])}")
            for et, c in blk.csr.items():
                rp.append(c.fwd.rowptr)
                col.append(c.fwd.col if c.num_edges else None)
                outer = h == L - 1
                mp.append(mb.nodes[0][et[0]] if outer else None)   # local -> global ids
                nd.append(c.n_dst)
                e.append(c.num_edges)
                rpo.append(self.rowptr[h][et])
                colo.append(self.col[h][et])
                dcap.append(self.cap[h][et[2]])
                ecap.append(self.ecap[h][et])
                # padding entries read source row 0 of the global table (outermost block: no
                # transposed grouping is built for it) or, in turn, the `slack` padded rows at
                # the end of the level-(h+1) table (its backward's CSC then has no long row)
                dummy.append(0 if outer else self.cap[h + 1][et[0]] - self.slack)
                spread.append(1 if outer else self.slack)
        for t, ids in self.root_ids.items():
            src = mb.nodes[1][t]                                   # level L - 1 (nodes reversed)
            rp.append(None)
            col.append(src if src.numel() else None)
            mp.append(None)
            nd.append(0)
            e.append(int(src.numel()))
            rpo.append(None)
            colo.append(ids)
            dcap.append(-1)
            ecap.append(int(ids.numel()))
            dummy.append(0)
            spread.append(1)
        n = len(rp)
        N.check(N.lib().hgnn_pad_csr_multi(
            n, N.ptr_array(rp), N.ptr_array(col), N.ptr_array(mp), N.i64_array(nd),
            N.i64_array(e), N.ptr_array(rpo), N.ptr_array(colo), N.i64_array(dcap),
            N.i64_array(ecap), N.int_array(dummy), N.int_array(spread),
            N.stream_ptr(self.smp.device)),
            "hgnn_pad_csr_multi")

    def make_csrs(self) -> None:
        """Fresh relation objects over the buffers (their CSC / 1/deg are built on first use:
        inside the graph when this runs right before capture)."""
        out = []
        for h in range(self.L):
            outer = h == self.L - 1
            csrs = {et: RelationCSR.from_csr(
                self.rowptr[h][et], self.col[h][et][:self.ecap[h][et]],
                self.smp.num_nodes[et[0]] if outer else self.cap[h + 1][et[0]],
                self.cap[h][et[2]], may_have_heavy_rows=False) for et in self.ecap[h]}
            group = [weakref.ref(c) for c in csrs.values()]
            for c in csrs.values():
                c._csc_group = group
            out.append(csrs)
        self.csrs = out

    # -- the model on the static blocks --------------------------------------------------------
    def forward(self, model: HeteroSAGE, x_dict: Mapping[str, torch.Tensor]
                ) -> Dict[str, torch.Tensor]:
        """``model`` on the static blocks; the seeds' rows per type (seed order), as
        ``sampler.forward_blocks`` returns them for the loaded batch."""
        if len(model.layers) != self.L:
            raise ValueError(f"{len(model.layers)}-layer model on {self.L} static levels")
        L = self.L
        # outermost block: relations gather the global tables; roots are their own input
        h_in = {t: x_dict[t] for t in self.smp.num_nodes}
        for t, ids in self.root_ids.items():
            h_in[f"{t}@root"] = x_dict[t].index_select(0, ids)
        h: Dict[str, torch.Tensor] = {}
        for li in range(L):
            hop = L - 1 - li
            convs, csrs = model.layers[li], self.csrs[hop]
            outer = li == 0
            out, groups, weights = {}, [], []
            for dst in sorted(self.cap[hop]):
                msgs = [("__".join(et), et, w) for et, w in model.relations
                        if et[2] == dst and et in csrs]
                if not msgs:
                    out[dst] = h_in[f"{dst}@root"] if outer else h[dst][:self.cap[hop][dst]]
                    continue
                rels = tuple((et[0], csrs[et]) for _, et, _ in msgs)
                if outer:
                    groups.append(ops.DstGroup(dst, rels, True, True, (), None,
                                               root_src=f"{dst}@root"))
                else:
                    groups.append(ops.DstGroup(dst, rels, True, True, (),
                                               n_root=self.cap[hop][dst]))
                weights.append(_fused_weights(convs, msgs, h_in if outer else h))
            src = h_in if outer else h
            if groups:
                out.update(ops.hetero_layer(ops.LayerSpec(tuple(sorted(src)), tuple(groups)), src,
                                            weights))
            h = out
        return {t: h[t][:n] for t, n in self.n_seeds.items()}


class CapturedStep:
    """Forward + ``loss_fn(out)`` + backward (+ ``optimizer.step()``) of a sampled mini-batch,
    captured once on static blocks and replayed per batch.  The optimizer must be capturable
    (``torch.optim.Adam(..., capturable=True)``); gradients live in the graph's memory pool and
    are rewritten by every replay (zeroed once before capture).

    ``between`` (data-parallel ranks): a call between the backward and the optimizer step —
    ``parallel.sync_grads``'s all-reduce of the gradients.  With ``capture_between`` (RCCL: its
    collectives are graph-capturable) it is recorded INSIDE the one graph, so a step is one
    replay; otherwise (gloo, whose collectives run on the host) it runs eagerly and the step is
    two replays, the forward + loss + backward graph and the optimizer graph, around it.  A
    ``loss_fn`` with a ``make_csr()`` method (``LinkLoss``) gets fresh structures before each
    recorded pass.

    ``partial_seeds`` (``StaticBlocks``): None takes the loss's own ``partial_seeds`` attribute
    (``LinkLoss`` sets it: it reads seed rows by local id), else False."""

    def __init__(self, model: HeteroSAGE, x_dict: Mapping[str, torch.Tensor],
                 smp: NeighborSampler, n_seeds: Mapping[str, int],
                 loss_fn: Callable[[Dict[str, torch.Tensor]], torch.Tensor],
                 optimizer: Optional[torch.optim.Optimizer] = None, slack: int = SLACK,
                 between: Optional[Callable[[], None]] = None,
                 partial_seeds: Optional[bool] = None, capture_between: bool = False):
        self.model, self.x_dict, self.loss_fn, self.opt = model, x_dict, loss_fn, optimizer
        self.between = between
        self.capture_between = bool(capture_between) and between is not None
        if self.capture_between:
            # a collective recorded into the graph must be a device-side one (RCCL); gloo runs
            # its collectives on the host and cannot be captured
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized() and dist.get_backend() != "nccl":
                raise ValueError("CapturedStep(capture_between=True) needs the nccl (RCCL) "
                                 f"backend; got {dist.get_backend()!r} — leave capture_between "
                                 "off to replay around an eager all-reduce")
        if partial_seeds is None:
            partial_seeds = bool(getattr(loss_fn, "partial_seeds", False))
        self.blocks = StaticBlocks(smp, n_seeds, slack, partial_seeds=partial_seeds)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.graph_opt: Optional[torch.cuda.CUDAGraph] = None
        self.loss: Optional[torch.Tensor] = None
        self.out: Optional[Dict[str, torch.Tensor]] = None

    def _fresh(self):
        self.blocks.make_csrs()
        mk = getattr(self.loss_fn, "make_csr", None)
        if mk is not None:
            mk()

    def _body(self, with_opt: bool = True):
        out = self.blocks.forward(self.model, self.x_dict)
        loss = self.loss_fn(out)
        loss.backward()
        if self.capture_between:
            self.between()
        if self.opt is not None and with_opt:
            self.opt.step()
        return out, loss

    def capture(self, first: MiniBatch, warmup: int = 2) -> None:
        """Warm up eagerly on ``first`` (library handles, allocator pools; with an optimizer
        these are training steps), then record the step."""
        dev = self.blocks.smp.device
        self.blocks.load(first)
        split = self.between is not None and self.opt is not None and not self.capture_between
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._fresh()
                self._zero_grad()
                self._body(with_opt=not split)
                if split:
                    self.between()
                    self.opt.step()
        torch.cuda.current_stream(dev).wait_stream(side)
        self._fresh()                      # fresh: their CSC and 1/deg builds are recorded
        self._zero_grad()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out, loss = self._body(with_opt=not split)
        # the static outputs without the recorded autograd graph (kept alive, its AccumulateGrad
        # nodes would tie later eager backwards of the same parameters to the capture stream)
        self.out = {t: v.detach() for t, v in out.items()}
        self.loss = loss.detach()
        del out, loss
        self.graph = g
        if split:
            go = torch.cuda.CUDAGraph()
            with torch.cuda.graph(go):
                self.opt.step()
            self.graph_opt = go

    def _zero_grad(self):
        if self.opt is not None:
            self.opt.zero_grad(set_to_none=True)
        else:
            self.model.zero_grad(set_to_none=True)

    def step(self, mb: MiniBatch) -> torch.Tensor:
        """``mb`` through the recorded step (queued, no sync); returns the static loss tensor."""
        if self.graph is None:
            raise RuntimeError("CapturedStep.step before capture()")
        self.blocks.load(mb)
        self.graph.replay()
        if self.graph_opt is not None:
            self.between()
            self.graph_opt.replay()
        return self.loss


# ----------------------------------------------------------------------------- link batches
class _LossCSR:
    """The grouping ``ops._edge_bce`` reads for a link batch: ``bwd`` = the positive pairs by
    user (built outside the step), ``fwd`` = the same pairs by post (the transposed grouping of
    a ``from_csr`` relation: one ``hgnn_csr_transpose`` on first use, no host sync)."""

    def __init__(self, rowptr_u, col_p, uop, n_users: int, n_posts: int):
        self._rel = RelationCSR.from_csr(rowptr_u, col_p, n_posts, n_users,
                                         may_have_heavy_rows=False)
        self.n_src, self.n_dst = int(n_users), int(n_posts)
        self.num_edges = int(col_p.numel())
        self._uop = uop

    @property
    def fwd(self):
        return self._rel.bwd

    @property
    def bwd(self):
        return self._rel.fwd


class LinkLoss:
    """The reference's loss (train_gnn.py:259-281: BCE-with-logits means over the positive
    edges and over one uniform negative post per positive, unit edge weights) on a link
    mini-batch, through the library's fused loss kernels (``ops._EdgeBCELoss``) over fixed-size
    buffers: ``load(pu, pp, pn)`` (local user / post ids of the positives, local post ids of the
    negatives; no sync) groups the pairs by user into them, ``make_csr()`` makes fresh
    structures over them (their post grouping is built on first use: inside a capture, per
    replay).  ``n_total`` = the positives of ALL ranks, so per-rank losses add up to the global
    batch's mean (data-parallel gradients are summed).  It reads the seed rows by local id, so
    a batch with fewer distinct endpoints than the capacity is fine (``partial_seeds``)."""

    partial_seeds = True

    def __init__(self, n_edges: int, n_users: int, n_posts: int, device, n_total: int = 0):
        i32 = dict(dtype=torch.int32, device=device)
        self.E, self.n_users, self.n_posts = int(n_edges), int(n_users), int(n_posts)
        self.n_total = int(n_total) if n_total else self.E
        self.rowptr = torch.zeros(self.n_users + 1, **i32)
        self.col = torch.zeros(self.E, **i32)
        self.neg = torch.zeros(self.E, **i32)
        self.uop = torch.zeros(self.E, **i32)
        self.cscale = torch.ones((), dtype=torch.float32, device=device)
        self.csr: Optional[_LossCSR] = None

    def load(self, pu: torch.Tensor, pp: torch.Tensor, pn: torch.Tensor) -> None:
        if int(pu.numel()) != self.E:
            raise ValueError(f"{int(pu.numel())} positives for a {self.E}-edge link loss")
        order = torch.argsort(pu, stable=True)
        cnt = torch.zeros(self.n_users + 1, dtype=torch.int64, device=pu.device)
        cnt.scatter_add_(0, pu.to(torch.int64) + 1, torch.ones_like(pu, dtype=torch.int64))
        self.rowptr.copy_(torch.cumsum(cnt, 0))
        self.col.copy_(pp[order])
        self.neg.copy_(pn[order])
        self.uop.copy_(pu[order])

    def make_csr(self) -> None:
        self.csr = _LossCSR(self.rowptr, self.col, self.uop, self.n_users, self.n_posts)

    def __call__(self, out: Mapping[str, torch.Tensor]) -> torch.Tensor:
        U, P = out["user"], out["post"]
        if int(U.shape[0]) != self.n_users or int(P.shape[0]) != self.n_posts:
            raise ValueError(f"link loss over {self.n_users} users / {self.n_posts} posts, got "
                             f"{tuple(U.shape)} / {tuple(P.shape)}")
        if self.csr is None:
            self.make_csr()
        return ops._EdgeBCELoss.apply(U, P, self.csr, self.neg, self.cscale, False, self.n_total)


@dataclasses.dataclass
class LinkBatch:
    """A link-prediction mini-batch (PyG LinkNeighborLoader semantics, binary negatives): B
    positive ``engages`` edges, one uniform negative post per positive (train_gnn.py:272), the
    seeds = the distinct endpoints (users; posts of the positives and negatives, each sorted),
    and the pairs as local ids into the seeds (= the sampled outputs' rows)."""
    pos_u: torch.Tensor      # global ids [B]
    pos_p: torch.Tensor
    neg_p: torch.Tensor
    seeds: Dict[str, torch.Tensor]
    pu: torch.Tensor         # local ids [B]
    pp: torch.Tensor
    pn: torch.Tensor
    mb: Optional[MiniBatch] = None


def link_batch(edge_index: torch.Tensor, edge_ids: torch.Tensor, num_posts: int,
               generator: Optional[torch.Generator] = None) -> LinkBatch:
    """The positives ``edge_index[:, edge_ids]`` ((user, post) rows), their negatives drawn
    uniformly over the posts, the distinct endpoints as seeds (two host syncs: the unique
    counts)."""
    pos_u, pos_p = edge_index[0, edge_ids], edge_index[1, edge_ids]
    neg_p = torch.randint(0, int(num_posts), (int(edge_ids.numel()),), device=pos_u.device,
                          generator=generator, dtype=pos_u.dtype)
    su = torch.unique(pos_u)
    sp = torch.unique(torch.cat([pos_p, neg_p]))
    return LinkBatch(pos_u, pos_p, neg_p, {"user": su, "post": sp},
                     torch.searchsorted(su, pos_u), torch.searchsorted(sp, pos_p),
                     torch.searchsorted(sp, neg_p))
