"""A neighbour-sampled mini-batch step replayed as one HIP graph (BASELINE cfg5).

``sampler.forward_blocks`` issues ~120 launches per step from Python and the autograd engine: at
cfg5 the step is bound by host issue (2.1 ms of host work per step against ~1.2 ms of GPU work,
``scripts/cfg5_breakdown.py``).  A graph needs fixed shapes, and every sampled batch has its own
node and edge counts, so this module runs the model on STATIC-CAPACITY blocks:

* capacities follow from the seeds and fanouts alone: level 0 holds the seeds, level h + 1 at
  most level h plus fanout x level-h destinations per relation out of each source type; every
  level gets ``slack`` padded rows on top (>= 1 padded destination row for the padding edges,
  and a padded source row for them to read);
* every per-batch input the graph reads lives in one byte arena (``_Arena``), held twice: the
  LIVE copy the graph was recorded on and a STAGE copy a batch is prepared into.
  ``prepare(batch)`` fills the stage — the block CSRs padded to capacity in ONE launch
  (``hgnn_pad_csr_multi``: real rows first and unchanged, the padding entries spread over the
  padded rows and pointing at a padded source row; the outermost block's column ids mapped to
  GLOBAL ids on the way, so its gathers read the feature tables directly), the outermost
  destinations' own rows (``DstGroup.root_src``) gathered from the feature tables, and the CSCs
  + per-position 1/deg of the inner blocks (one ``hgnn_csr_transpose_multi``) that the backward
  needs; ``commit()`` is ONE device copy stage -> live.  So the structure builds run on whatever
  stream ``prepare`` is called on — a side stream under the previous replay, next to the
  sampler — and the replay itself is the model's kernels only (round 6: 28 fewer graph nodes);
* ``capture(loss_fn, optimizer)`` records forward + loss + backward (+ the optimizer step) once;
  ``step(batch)`` = ``prepare`` + ``commit`` + replay (``step()`` after a ``prepare`` elsewhere).

Padded rows carry finite junk (means of padded source rows) that never reaches a seed: a padded
destination row is never a source of a real row, and the loss reads the seed rows only, so the
padded rows' gradients are exactly 0 and add nothing to the weight gradients.  Tested against
the eager ``forward_blocks`` step on the same batches (outputs, loss, every parameter gradient).
"""
from __future__ import annotations

import dataclasses
from typing import Callable, Dict, List, Mapping, Optional, Tuple

import torch

from . import _native as N
from . import ops
from .graph import NO_SPLIT, GroupedEdges, Plan, RelationCSR
from .nn import HeteroSAGE, _fused_weights_layers
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


class _Arena:
    """Named per-batch buffers in one byte arena, held twice with one layout: ``live`` (what a
    recorded graph reads) and ``stage`` (where the next batch is written, on any stream).
    ``commit()`` = one device copy stage -> live on the current stream; ``prepare`` callers wait
    for the last commit first (``wait_committed``), so a stage write never races the copy that
    reads it.  Offsets are 256-byte aligned; both copies start zeroed (a valid empty CSR)."""

    ALIGN = 256

    def __init__(self, specs: Mapping[str, Tuple[int, torch.dtype]], device):
        self.layout, off = {}, 0
        for k, (n, dt) in specs.items():
            nb = int(n) * torch.empty((), dtype=dt).element_size()
            self.layout[k] = (off, int(n), dt, nb)
            off += -(-max(nb, 1) // self.ALIGN) * self.ALIGN
        self.nbytes = off
        self._bytes = {w: torch.zeros(max(off, self.ALIGN), dtype=torch.uint8, device=device)
                       for w in ("live", "stage")}
        self.live = self._views("live")
        self.stage = self._views("stage")
        self._committed: Optional[torch.cuda.Event] = None
        self._dirty = False
        # direct: writers fill the LIVE buffers themselves (two captured steps replayed in turn,
        # each batch prepared into the one not replaying); commit() copies nothing, and the
        # event a writer waits for is the last replay that read them (consumed())
        self.direct = False

    def _views(self, which):
        buf = self._bytes[which]
        return {k: buf[o:o + nb].view(dt) for k, (o, n, dt, nb) in self.layout.items()}

    def wait_committed(self) -> None:
        """Called by a writer of the stage before it writes (on its stream)."""
        if self._committed is not None:
            torch.cuda.current_stream(self._bytes["stage"].device).wait_event(self._committed)
        self._dirty = True

    def target(self):
        """The buffers a writer fills: the stage, or the live ones in direct mode."""
        return self.live if self.direct else self.stage

    def consumed(self) -> None:
        """Direct mode: the live buffers were just read (a replay was queued on the current
        stream); the next writer waits for this point."""
        ev = torch.cuda.Event()
        ev.record()
        self._committed = ev

    def commit(self) -> None:
        """No-op when nothing was prepared since the last commit (and in direct mode)."""
        if not self._dirty or self.direct:
            self._dirty = False
            return
        self._dirty = False
        self._bytes["live"].copy_(self._bytes["stage"])
        if self._bytes["live"].is_cuda:
            ev = torch.cuda.Event()
            ev.record()
            self._committed = ev


class StaticBlocks:
    """Fixed-capacity buffers for the blocks of one sampler configuration (see module doc).

    ``x_dict``: the feature tables the outermost block reads (their rows per type give the
    staged root rows' width).  ``partial_seeds``: a batch may hold FEWER seeds than ``n_seeds``
    (the rest are padded level-0 rows).  Only a loss that reads the seed rows by their local ids
    may allow it (``LinkLoss``: a link batch's distinct endpoints vary in number); a loss over
    all seed rows would be fed the padding, so by default a batch must have exactly ``n_seeds``
    seeds per type."""

    def __init__(self, smp: NeighborSampler, n_seeds: Mapping[str, int],
                 x_dict: Mapping[str, torch.Tensor], slack: int = SLACK,
                 partial_seeds: bool = False):
        self.smp = smp
        self.x_dict = x_dict
        self.n_seeds = {t: int(n) for t, n in n_seeds.items()}
        self.partial_seeds = bool(partial_seeds)
        if slack < 1:
            raise ValueError("slack: at least one padded row per level")
        self.slack = int(slack)
        self.L = len(smp.fanouts)
        self.cap, self.ecap = capacities(smp.relations, self.n_seeds, smp.fanouts, slack)
        if max(max(c.values()) for c in self.cap) >= 2**31 - 1:
            raise ValueError("static block capacities exceed int32")
        L, i32, f32 = self.L, torch.int32, torch.float32
        spec: Dict[str, Tuple[int, torch.dtype]] = {}
        for h in range(L):
            for et in self.ecap[h]:
                E = max(self.ecap[h][et], 1)
                spec[f"rp{h}{et}"] = (self.cap[h][et[2]] + 1, i32)
                spec[f"col{h}{et}"] = (E, i32)
                if h < L - 1:
                    # the inner blocks' CSC + K2 weights (the outermost block reads the feature
                    # tables, which take no gradient: it has no backward gather)
                    spec[f"crp{h}{et}"] = (self.cap[h + 1][et[0]] + 1, i32)
                    spec[f"ccol{h}{et}"] = (E, i32)
                    spec[f"cperm{h}{et}"] = (E, i32)
                    spec[f"cw{h}{et}"] = (E, f32)
        # the outermost block's destinations (level L - 1): global ids and their feature rows
        for t, n in self.cap[L - 1].items():
            spec[f"root_ids{t}"] = (n, i32)
            spec[f"root_x{t}"] = (n * int(x_dict[t].shape[1]), x_dict[t].dtype)
        self.arena = _Arena(spec, smp.device)
        self.csrs: Optional[List[Dict[EdgeType, RelationCSR]]] = None
        self._static_calls()

    def use_direct(self) -> None:
        """Prepare straight into the live buffers (``_Arena.direct``): for two captured steps
        replayed in turn, each batch staged into the one that is not replaying."""
        self.arena.direct = True
        self._static_calls()

    def _static_calls(self) -> None:
        """The staging calls' arguments that do not change per batch (the target buffers, the
        capacities), built once: a batch then fills five small arrays (its CSR and id
        pointers, row and entry counts) — prepare's host cost is three ctypes calls."""
        L, st, dev = self.L, self.arena.target(), self.smp.device
        lib = N.lib()
        # pad items: every (hop, relation) in the static layout's order, then the root id lists
        self._items = [(h, et) for h in range(L) for et in self.ecap[h]]
        roots = list(self.cap[L - 1])
        n = len(self._items) + len(roots)
        if n > 16:
            raise ValueError(f"{n} padded items: hgnn_pad_csr_multi takes at most 16")
        outer = [h == L - 1 for h, _ in self._items]
        self._pad_var = [(N._p * n)(), (N._p * n)(), (N._p * n)(), (N._c_i64 * n)(),
                         (N._c_i64 * n)()]                     # rowptr, col, map, n_dst, E
        self._pad_static = (
            N.ptr_array([st[f"rp{h}{et}"] for h, et in self._items] + [None] * len(roots)),
            N.ptr_array([st[f"col{h}{et}"] for h, et in self._items]
                        + [st[f"root_ids{t}"] for t in roots]),
            N.i64_array([self.cap[h][et[2]] for h, et in self._items] + [-1] * len(roots)),
            N.i64_array([self.ecap[h][et] for h, et in self._items]
                        + [self.cap[L - 1][t] for t in roots]),
            # padding entries read source row 0 of the global table (outermost block: no
            # transposed grouping is built for it) or, in turn, the `slack` padded rows at the
            # end of the level-(h+1) table (its backward's CSC then has no long row)
            N.int_array([0 if o else self.cap[h + 1][et[0]] - self.slack
                         for (h, et), o in zip(self._items, outer)] + [0] * len(roots)),
            N.int_array([1 if o else self.slack for o in outer] + [1] * len(roots)))
        self._n_pad = n
        # the root rows: one gather of every type's rows
        dims = {int(self.x_dict[t].shape[1]) for t in roots}
        if len(dims) != 1 or any(self.x_dict[t].dtype != torch.float32 for t in roots):
            raise ValueError("static blocks: the feature tables must be fp32 of one width")
        self._rows_args = (len(roots), N.ptr_array([self.x_dict[t] for t in roots]),
                           N.ptr_array([st[f"root_ids{t}"] for t in roots]),
                           N.i64_array([self.cap[L - 1][t] for t in roots]), dims.pop(),
                           N.ptr_array([st[f"root_x{t}"] for t in roots]))
        # the inner blocks' CSCs: one hgnn_csr_transpose_multi per inner hop, static workspace
        self._csc_args = []
        for h in range(L - 1):
            ets = list(self.ecap[h])
            Es = [self.ecap[h][et] for et in ets]
            ncols = [self.cap[h + 1][et[0]] for et in ets]
            ws = torch.empty(max(int(lib.hgnn_csr_transpose_multi_ws_bytes(sum(Es), sum(ncols))),
                                 256), dtype=torch.uint8, device=dev)
            self._csc_args.append((ws, (
                len(ets), N.ptr_array([st[f"rp{h}{et}"] for et in ets]),
                N.ptr_array([st[f"col{h}{et}"] for et in ets]),
                N.i64_array([self.cap[h][et[2]] for et in ets]), N.i64_array(Es),
                N.i64_array(ncols), N.ptr_array([st[f"crp{h}{et}"] for et in ets]),
                N.ptr_array([st[f"ccol{h}{et}"] for et in ets]),
                N.ptr_array([st[f"cperm{h}{et}"] for et in ets]),
                N.ptr_array([st[f"cw{h}{et}"] for et in ets]), ws.data_ptr(), ws.numel())))

    def rowptr(self, h: int, et: EdgeType, which: str = "live") -> torch.Tensor:
        return getattr(self.arena, which)[f"rp{h}{et}"]

    def col(self, h: int, et: EdgeType, which: str = "live") -> torch.Tensor:
        return getattr(self.arena, which)[f"col{h}{et}"][:self.ecap[h][et]]

    def root_rows(self, t: str, which: str = "live") -> torch.Tensor:
        return getattr(self.arena, which)[f"root_x{t}"].view(self.cap[self.L - 1][t], -1)

    # -- per batch ---------------------------------------------------------------------------
    def prepare(self, mb: MiniBatch) -> None:
        """The batch into the STAGE buffers on the current stream (no sync): the padded CSRs
        and root ids (one launch), the root rows (one launch) and the inner blocks' CSCs (one
        launch per inner hop).  ``commit()`` makes them the live ones."""
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
        rp, col, mp, nd, e = self._pad_var
        for i, (h, et) in enumerate(self._items):
            blk = mb.blocks[L - 1 - h]
            c = blk.csr.get(et)
            if c is None or len(blk.csr) != len(self.ecap[h]):
                raise ValueError(f"hop {h}: relations {sorted(blk.csr)} differ from the static "
                                 f"layout {sorted(self.ecap[h])}")
            rp[i] = c.fwd.rowptr.data_ptr()
            col[i] = c.fwd.col.data_ptr() if c.num_edges else None
            # the outermost block's local source ids -> global ids
            mp[i] = mb.nodes[0][et[0]].data_ptr() if h == L - 1 else None
            nd[i] = c.n_dst
            e[i] = c.num_edges
        for i, t in enumerate(self.cap[L - 1], len(self._items)):
            src = mb.nodes[1][t]                                   # level L - 1 (nodes reversed)
            rp[i] = mp[i] = None
            col[i] = src.data_ptr() if src.numel() else None
            nd[i] = 0
            e[i] = int(src.numel())
        self.arena.wait_committed()
        lib, s = N.lib(), N.stream_ptr(self.smp.device)
        rpo, colo, dcap, ecap, dummy, spread = self._pad_static
        N.check(lib.hgnn_pad_csr_multi(self._n_pad, rp, col, mp, nd, e, rpo, colo, dcap, ecap,
                                       dummy, spread, s), "hgnn_pad_csr_multi")
        self._stage_derived(lib, s)

    def _stage_derived(self, lib, s) -> None:
        """What follows from the staged CSRs and root ids: the root rows and the CSCs."""
        N.check(lib.hgnn_gather_rows_multi(*self._rows_args, s), "hgnn_gather_rows_multi")
        for _, args in self._csc_args:
            N.check(lib.hgnn_csr_transpose_multi(*args, s), "hgnn_csr_transpose_multi")

    def commit(self) -> None:
        """The prepared batch becomes the live one: one device copy on the current stream."""
        self.arena.commit()

    def load(self, mb: MiniBatch) -> None:
        """``prepare`` + ``commit`` on the current stream."""
        self.prepare(mb)
        self.commit()

    def make_csrs(self) -> None:
        """Relation objects over the LIVE buffers, their CSCs and K2 weights set to the live
        ones (nothing of them is built inside a recorded step)."""
        out, lv = [], self.arena.live
        for h in range(self.L):
            outer = h == self.L - 1
            csrs = {}
            for et in self.ecap[h]:
                n_src = self.smp.num_nodes[et[0]] if outer else self.cap[h + 1][et[0]]
                E = self.ecap[h][et]
                c = RelationCSR.from_csr(self.rowptr(h, et), self.col(h, et), n_src,
                                         self.cap[h][et[2]], may_have_heavy_rows=False)
                if not outer:
                    c._bwd = GroupedEdges(lv[f"crp{h}{et}"], lv[f"ccol{h}{et}"][:E],
                                          lv[f"cperm{h}{et}"][:E],
                                          Plan(NO_SPLIT, 0, 0, None, None), n_src)
                    c._bwd_w = lv[f"cw{h}{et}"][:E]
                csrs[et] = c
            out.append(csrs)
        self.csrs = out

    # -- the model on the static blocks --------------------------------------------------------
    def forward(self, model: HeteroSAGE, x_dict: Mapping[str, torch.Tensor],
                padded: bool = False) -> Dict[str, torch.Tensor]:
        """``model`` on the static blocks; the seeds' rows per type (seed order), as
        ``sampler.forward_blocks`` returns them for the loaded batch — or, ``padded``, the whole
        level-0 tables (``cap[0]`` rows: the seeds, then padded rows) for a loss that reads rows
        by id and gives the others a zero gradient (no slice, so no zero-fill + copy of its
        backward)."""
        if len(model.layers) != self.L:
            raise ValueError(f"{len(model.layers)}-layer model on {self.L} static levels")
        L = self.L
        if any(x_dict[t] is not v for t, v in self.x_dict.items()):
            raise ValueError("StaticBlocks.forward: other feature tables than the staged root "
                             "rows were gathered from")
        # outermost block: relations gather the global tables; roots are their own input
        h_in = {t: x_dict[t] for t in self.smp.num_nodes}
        for t in self.cap[L - 1]:
            h_in[f"{t}@root"] = self.root_rows(t)
        h: Dict[str, torch.Tensor] = {}
        # every layer's fused weights in one launch (and their split in one): the weights do
        # not depend on the activations, only each layer's input widths
        layer_msgs = []
        for li in range(L):
            csrs = self.csrs[L - 1 - li]
            msgs_g = [m for m in ([("__".join(et), et, w) for et, w in model.relations
                                   if et[2] == dst and et in csrs]
                                  for dst in sorted(self.cap[L - 1 - li])) if m]
            dims = ({t: int(x.shape[1]) for t, x in x_dict.items()} if li == 0 else
                    {t: int(model.hidden_dim) for t in self.smp.num_nodes})
            layer_msgs.append((model.layers[li], msgs_g, dims))
        weights_all = _fused_weights_layers(layer_msgs)
        for li in range(L):
            hop = L - 1 - li
            convs, csrs = model.layers[li], self.csrs[hop]
            outer = li == 0
            out, groups = {}, []
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
            src = h_in if outer else h
            if groups:
                out.update(ops.hetero_layer(ops.LayerSpec(tuple(sorted(src)), tuple(groups)), src,
                                            weights_all[li]))
            h = out
        if padded:
            return {t: h[t] for t in self.n_seeds}
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
        self.blocks = StaticBlocks(smp, n_seeds, x_dict, slack, partial_seeds=partial_seeds)
        self._unit = ops.unit_grad(smp.device)
        # a loss that takes the padded level-0 tables (LinkLoss) is sized for them here
        pad = getattr(loss_fn, "use_padded_rows", None)
        self.padded = pad is not None
        if self.padded:
            pad({t: self.blocks.cap[0][t] for t in self.blocks.n_seeds})
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
        out = self.blocks.forward(self.model, self.x_dict, padded=self.padded)
        loss = self.loss_fn(out)
        loss.backward(self._unit)          # a marked 1: no fill, no scale-by-1 launches
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
        self._fresh()
        self._zero_grad()
        g = torch.cuda.CUDAGraph(keep_graph=True)   # kept: its nodes are counted (graph_nodes)
        with torch.cuda.graph(g):
            out, loss = self._body(with_opt=not split)
        g.instantiate()
        # the static outputs without the recorded autograd graph (kept alive, its AccumulateGrad
        # nodes would tie later eager backwards of the same parameters to the capture stream)
        self.out = {t: v.detach() for t, v in out.items()}
        self.loss = loss.detach()
        del out, loss
        self.graph = g
        if split:
            go = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.graph(go):
                self.opt.step()
            go.instantiate()
            self.graph_opt = go

    def graph_nodes(self) -> Optional[Dict[str, int]]:
        """Nodes of the recorded step's graph(s) by kind (hipGraphGetNodes /
        hipGraphNodeGetType): kernels, copies, memsets, other."""
        if self.graph is None:
            return None
        return _graph_node_counts([g for g in (self.graph, self.graph_opt) if g is not None])

    def _zero_grad(self):
        if self.opt is not None:
            self.opt.zero_grad(set_to_none=True)
        else:
            self.model.zero_grad(set_to_none=True)

    def prepare(self, mb: MiniBatch, *loss_args) -> None:
        """The next batch into the staging buffers on the current stream (a side stream under
        the running replay, say): the blocks, and ``loss_fn.prepare(*loss_args)`` if given."""
        self.blocks.prepare(mb)
        if loss_args:
            self.loss_fn.prepare(*loss_args)

    def step(self, mb: Optional[MiniBatch] = None) -> torch.Tensor:
        """One recorded step (queued, no sync) on ``mb`` — or, with no argument, on the batch
        last ``prepare``d: the staged inputs committed (one copy each for the blocks and a
        loss with a ``commit``), then the replay.  Returns the static loss tensor."""
        if self.graph is None:
            raise RuntimeError("CapturedStep.step before capture()")
        if mb is not None:
            self.blocks.prepare(mb)
        self.blocks.commit()
        commit = getattr(self.loss_fn, "commit", None)
        if commit is not None:
            commit()
        self.graph.replay()
        if self.graph_opt is not None:
            self.between()
            self.graph_opt.replay()
        lf = getattr(self.loss_fn, "link_loss", self.loss_fn)    # (a wrapper's LinkLoss)
        for ar in (self.blocks.arena, getattr(lf, "arena", None)):
            if isinstance(ar, _Arena) and ar.direct:
                ar.consumed()
        return self.loss


def _graph_node_counts(graphs) -> Dict[str, int]:
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    kinds = {0: "kernel", 1: "memcpy", 2: "memset"}
    out = {"total": 0, "kernel": 0, "memcpy": 0, "memset": 0, "other": 0}
    for g in graphs:
        raw = ctypes.c_void_p(g.raw_cuda_graph())
        n = ctypes.c_size_t(0)
        if hip.hipGraphGetNodes(raw, None, ctypes.byref(n)) != 0:
            raise RuntimeError("hipGraphGetNodes failed")
        nodes = (ctypes.c_void_p * max(n.value, 1))()
        if hip.hipGraphGetNodes(raw, nodes, ctypes.byref(n)) != 0:
            raise RuntimeError("hipGraphGetNodes failed")
        for i in range(n.value):
            kind = ctypes.c_int(-1)
            hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(kind))
            out[kinds.get(kind.value, "other")] += 1
        out["total"] += n.value
    return out


# ----------------------------------------------------------------------------- link batches
class _LossCSR:
    """The groupings ``ops._edge_bce`` reads for a link batch, over a ``LinkLoss``'s live
    buffers: ``bwd`` = the positive pairs by user, ``fwd`` = the same pairs by post (the staged
    transpose; nothing is built inside a recorded step)."""

    def __init__(self, lv, n_users: int, n_posts: int):
        E = int(lv["col"].numel())
        self._rel = RelationCSR.from_csr(lv["rowptr"], lv["col"], n_posts, n_users,
                                         may_have_heavy_rows=False)
        self._rel._bwd = GroupedEdges(lv["p_rowptr"], lv["p_users"], lv["p_perm"],
                                      Plan(NO_SPLIT, 0, 0, None, None), n_posts)
        self.n_src, self.n_dst = int(n_users), int(n_posts)
        self.num_edges = E
        self._uop = lv["uop"]

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
    buffers (an ``_Arena``, live + stage, as ``StaticBlocks``).  ``prepare(pu, pp, pn)`` (local
    user / post ids of the positives, local post ids of the negatives; no sync) writes the
    stage in one call (``hgnn_link_group``): the pairs grouped by user, the same pairs grouped
    by post and the negatives grouped by post (the dP gather's order) — every structure the
    loss needs, so none is built inside a recorded step; ``commit()`` makes them live (one
    copy); ``load`` = both.  ``n_total`` = the positives of ALL ranks, so per-rank
    losses add up to the global batch's mean (data-parallel gradients are summed).  It reads the
    seed rows by local id, so a batch with fewer distinct endpoints than the capacity is fine
    (``partial_seeds``)."""

    partial_seeds = True

    def __init__(self, n_edges: int, n_users: int, n_posts: int, device, n_total: int = 0):
        self.E, self.n_users, self.n_posts = int(n_edges), int(n_users), int(n_posts)
        self.n_total = int(n_total) if n_total else self.E
        self.device = torch.device(device)
        self.cscale = torch.ones((), dtype=torch.float32, device=self.device)
        self._alloc(self.n_users, self.n_posts)

    def use_padded_rows(self, rows: Mapping[str, int]) -> None:
        """Take the embeddings as tables of ``rows`` (>= the id capacities) rows — a captured
        step's padded level-0 tables: the rows past the ids are empty groups whose gradient the
        loss writes as 0.  Called by ``CapturedStep`` before anything is loaded."""
        if rows["user"] < self.n_users or rows["post"] < self.n_posts:
            raise ValueError(f"padded rows {dict(rows)} below the id capacities")
        self._alloc(int(rows["user"]), int(rows["post"]))

    def use_direct(self) -> None:
        """Prepare straight into the live buffers (see ``StaticBlocks.use_direct``)."""
        self.arena.direct = True
        st = self.arena.target()
        self._stage_ptrs = tuple(st[k].data_ptr() for k in (
            "rowptr", "col", "neg", "uop", "p_rowptr", "p_users", "p_perm", "n_rowptr",
            "n_users"))

    def _alloc(self, rows_u: int, rows_p: int) -> None:
        i32, E = torch.int32, self.E
        self.rows = {"user": rows_u, "post": rows_p}
        self.arena = _Arena({"rowptr": (rows_u + 1, i32), "col": (E, i32),
                             "neg": (E, i32), "uop": (E, i32),
                             "p_rowptr": (rows_p + 1, i32), "p_users": (E, i32),
                             "p_perm": (E, i32), "n_rowptr": (rows_p + 1, i32),
                             "n_users": (E, i32)}, self.device)
        self.csr: Optional[_LossCSR] = None
        self.presorted = None
        st = self.arena.stage
        self._stage_ptrs = tuple(st[k].data_ptr() for k in (
            "rowptr", "col", "neg", "uop", "p_rowptr", "p_users", "p_perm", "n_rowptr",
            "n_users"))
        self._ws = torch.empty(max(int(N.lib().hgnn_link_group_ws_bytes(self.E)), 256),
                               dtype=torch.uint8, device=self.device)

    # the live buffers under their round-5 names
    rowptr = property(lambda self: self.arena.live["rowptr"])
    col = property(lambda self: self.arena.live["col"])
    neg = property(lambda self: self.arena.live["neg"])
    uop = property(lambda self: self.arena.live["uop"])

    def prepare(self, pu: torch.Tensor, pp: torch.Tensor, pn: torch.Tensor) -> None:
        if int(pu.numel()) != self.E:
            raise ValueError(f"{int(pu.numel())} positives for a {self.E}-edge link loss")
        pu, pp, pn = (t.to(torch.int32).contiguous() for t in (pu, pp, pn))
        self.arena.wait_committed()
        N.check(N.lib().hgnn_link_group(
            N.ptr(pu), N.ptr(pp), N.ptr(pn), self.E, self.rows["user"], self.rows["post"],
            *self._stage_ptrs, self._ws.data_ptr(), self._ws.numel(),
            N.stream_ptr(self.device)), "hgnn_link_group")

    def commit(self) -> None:
        self.arena.commit()

    def load(self, pu: torch.Tensor, pp: torch.Tensor, pn: torch.Tensor) -> None:
        self.prepare(pu, pp, pn)
        self.commit()

    def make_csr(self) -> None:
        lv = self.arena.live
        nu, np_ = self.rows["user"], self.rows["post"]
        self.csr = _LossCSR(lv, nu, np_)
        self.presorted = ops.PresortedNegatives(self.csr, lv["neg"], "user", np_,
                                                lv["n_rowptr"], lv["n_users"])

    def __call__(self, out: Mapping[str, torch.Tensor]) -> torch.Tensor:
        U, P = out["user"], out["post"]
        nu, np_ = self.rows["user"], self.rows["post"]
        if int(U.shape[0]) != nu or int(P.shape[0]) != np_:
            raise ValueError(f"link loss over {nu} user rows / {np_} post rows, got "
                             f"{tuple(U.shape)} / {tuple(P.shape)}")
        if self.csr is None:
            self.make_csr()
        return ops._EdgeBCELoss.apply(U, P, self.csr, self.arena.live["neg"], self.cscale,
                                      False, self.n_total, None,
                                      self.presorted if self.E else None)


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
    pu: torch.Tensor         # local ids [B] (int32)
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


class LinkSampler:
    """Link mini-batches sampled straight into a ``CapturedStep``'s staging buffers with no host
    sync (``csrc/sampler_static.hip``): per batch the negatives (the draws ``link_batch`` makes),
    the seeds and pair ids (``hgnn_link_seeds``), each hop over the static capacities with the
    counts kept on the device (``hgnn_sample_hop_static``; the inner hops relabelled by
    ``hgnn_relabel_static`` into the next frontier, the outermost hop's sources left as global
    ids), then the root rows, CSCs and loss groupings as ``prepare`` makes them.  The staged
    bytes equal ``link_batch`` + ``NeighborSampler.sample`` + ``CapturedStep.prepare`` on the
    same edges, draws and seed (tested), so the replayed step is unchanged; the host only
    queues ~10 calls (the eager sampler's read-backs made the host loop the
    cfg5 bound).  ``edge_ids``: the batch's positive edges into ``edge_index`` (int64 [B])."""

    def __init__(self, step: CapturedStep, edge_index: torch.Tensor, num_posts: int,
                 loss: Optional["LinkLoss"] = None):
        blocks = step.blocks
        loss = step.loss_fn if loss is None else loss     # the LinkLoss the step's loss reads
        smp = blocks.smp
        if not isinstance(getattr(loss, "arena", None), _Arena) or not hasattr(loss, "n_users"):
            raise ValueError("LinkSampler stages a LinkLoss (its loss_fn)")
        if set(blocks.n_seeds) != {"user", "post"} or blocks.n_seeds["post"] != 2 * loss.E \
                or blocks.n_seeds["user"] != loss.E:
            raise ValueError("LinkSampler: seeds capacities must be B users and 2B posts")
        if blocks.L < 2:
            raise ValueError("LinkSampler: at least two layers (the outermost block's "
                             "destinations are an inner hop's relabelled frontier)")
        self.step, self.blocks, self.loss = step, blocks, loss
        self.edge_index, self.num_posts, self.B = edge_index, int(num_posts), loss.E
        dev, i32, L = smp.device, torch.int32, blocks.L
        lib = N.lib()
        B = self.B
        self.seeds = {"user": torch.zeros(B, dtype=i32, device=dev),
                      "post": torch.zeros(2 * B, dtype=i32, device=dev)}
        self.pairs = torch.zeros(3, B, dtype=i32, device=dev)          # pu, pp, pn
        self.zero = torch.zeros(2, dtype=i32, device=dev)
        # per level: node counts per type (level 0: the seed kernel's [users, posts])
        self.counts = [torch.zeros(max(len(blocks.cap[h]), 2), dtype=i32, device=dev)
                       for h in range(L)]
        self.d_E = torch.zeros(L, 8, dtype=i32, device=dev)
        st = blocks.arena.target()      # (the live buffers when the blocks are in direct mode)
        # level h's node buffers (h >= 1): the outermost block's destinations are the staged
        # root ids; deeper inner levels a scratch buffer each
        nodes = [dict(self.seeds)]
        for h in range(1, L):
            nodes.append({t: st[f"root_ids{t}"] if h == L - 1
                          else torch.zeros(blocks.cap[h][t], dtype=i32, device=dev)
                          for t in blocks.cap[h]})
        self._nodes = nodes

        def cnt(h, t):          # device address of level h's count of type t
            if h == 0:
                return self.counts[0][0 if t == "user" else 1]
            return self.counts[h][sorted(blocks.cap[h]).index(t)]
        self._hops = []
        for h, fanout in enumerate(smp.fanouts):
            lvl = set(blocks.cap[h])
            types_h = sorted(lvl | {et[0] for et in smp.relations if et[2] in lvl})
            ets = sorted((et for et in smp.relations if et[2] in lvl),
                         key=lambda et: types_h.index(et[0]))
            outer = h == L - 1
            g = [smp.csr[et].fwd for et in ets]
            caps = [blocks.cap[h][et[2]] for et in ets]
            ecaps = [blocks.ecap[h][et] for et in ets]
            items = None if outer else torch.zeros(max(sum(ecaps), 1), dtype=i32, device=dev)
            fill = ([st[f"col{h}{et}"] for et in ets] if outer else
                    [items[o:o + c] for o, c in zip(_offsets(ecaps), ecaps)])
            ws = torch.empty(max(int(lib.hgnn_sample_hop_ws_bytes(sum(caps))), 256),
                             dtype=torch.uint8, device=dev)
            d_E = self.d_E[h]
            hop = dict(ws=ws, items=items, fanout=fanout, args=(
                len(ets), N.ptr_array([x.rowptr for x in g]), N.ptr_array([x.col for x in g]),
                N.i64_array([x.n_rows for x in g]),
                N.ptr_array([nodes[h][et[2]] for et in ets]),
                N.ptr_array([cnt(h, et[2]) for et in ets]), N.i64_array(caps),
                N.i64_array(ecaps)), outs=(
                N.ptr_array([st[f"rp{h}{et}"] for et in ets]), N.ptr_array(fill),
                N.ptr_array([st[f"col{h}{et}"] for et in ets]),
                N.int_array([0 if outer else blocks.cap[h + 1][et[0]] - blocks.slack
                             for et in ets]),
                N.int_array([1 if outer else blocks.slack for et in ets]), d_E.data_ptr(),
                ws.data_ptr(), ws.numel()))
            if not outer:
                nxt = sorted(blocks.cap[h + 1])
                if nxt != types_h:
                    raise ValueError(f"level {h + 1} types {nxt} differ from the hop's {types_h}")
                pcaps = [int(nodes[h][t].numel()) if t in lvl else 0 for t in types_h]
                rws = torch.empty(max(int(lib.hgnn_relabel_static_ws_bytes(sum(pcaps),
                                                                           sum(ecaps))), 256),
                                  dtype=torch.uint8, device=dev)
                hop["rws"] = rws
                hop["relabel"] = (
                    len(types_h),
                    N.ptr_array([nodes[h][t] if t in lvl else self.zero for t in types_h]),
                    N.ptr_array([cnt(h, t) if t in lvl else self.zero for t in types_h]),
                    N.i64_array(pcaps), N.ptr_array([nodes[h + 1][t] for t in types_h]),
                    N.i64_array([blocks.cap[h + 1][t] for t in types_h]), len(ets),
                    items.data_ptr(), N.i64_array(ecaps),
                    N.int_array([types_h.index(et[0]) for et in ets]), d_E.data_ptr(),
                    N.ptr_array([st[f"col{h}{et}"] for et in ets]),
                    self.counts[h + 1].data_ptr(), rws.data_ptr(), rws.numel())
            self._hops.append(hop)

    def prepare(self, edge_ids: torch.Tensor, seed: int,
                generator: Optional[torch.Generator] = None) -> None:
        """Batch ``seed``'s positives ``edge_ids`` into the staging buffers on the current
        stream (no sync); ``CapturedStep.step()`` then commits and replays it."""
        if int(edge_ids.numel()) != self.B:
            raise ValueError(f"{int(edge_ids.numel())} positives for a {self.B}-pair batch")
        dev = self.blocks.smp.device
        eid = edge_ids.to(torch.int64).contiguous()
        # the negatives exactly as link_batch draws them (same generator, same call)
        neg = torch.randint(0, self.num_posts, (self.B,), device=dev, generator=generator,
                            dtype=self.edge_index.dtype)
        self.blocks.arena.wait_committed()
        lib, s = N.lib(), N.stream_ptr(dev)
        ei = self.edge_index
        pu, pp, pn = self.pairs
        N.check(lib.hgnn_link_seeds(N.ptr(ei[0]), N.ptr(ei[1]), N.ptr(eid), N.ptr(neg), self.B,
                                    N.ptr(self.seeds["user"]), N.ptr(self.seeds["post"]),
                                    N.ptr(pu), N.ptr(pp), N.ptr(pn), N.ptr(self.counts[0]), s),
                "hgnn_link_seeds")
        for h, hop in enumerate(self._hops):
            hop_seed = (int(seed) * 1_000_003 + h) & 0xFFFFFFFFFFFFFFFF   # NeighborSampler's
            N.check(lib.hgnn_sample_hop_static(*hop["args"], hop["fanout"], hop_seed,
                                               *hop["outs"], s), "hgnn_sample_hop_static")
            if "relabel" in hop:
                N.check(lib.hgnn_relabel_static(*hop["relabel"], s), "hgnn_relabel_static")
        self.blocks._stage_derived(lib, s)
        self.loss.prepare(pu, pp, pn)

    def edge_count(self) -> torch.Tensor:
        """The staged batch's sampled message edges (every hop and relation), on the device."""
        return self.d_E.sum(dtype=torch.int64)


def _offsets(sizes):
    out, o = [], 0
    for n in sizes:
        out.append(o)
        o += n
    return out
