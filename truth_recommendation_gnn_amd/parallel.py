"""Multi-GPU hetero-SAGE: destination-partitioned, one process per GPU over RCCL.

One process per GPU (``torch.distributed``, backend ``nccl`` = RCCL over xGMI).  The user <-> post
graph is partitioned by USER (contiguous id ranges, the 10x larger node type), and the post
TABLE by row slices (``UserShard`` has the per-relation placement):

* post -> user relations (``rev_engages``): edges into owned users, read the all-gathered post
  table — complete on the owner, no exchange;
* user -> user relations (``social``): edges into owned users; the remote source rows (the halo)
  arrive by one all-to-all per layer with static split sizes, and their gradients go back by the
  reverse all-to-all;
* user -> post relations (``engages``): a per-rank PARTIAL sum over the rank's edges, each edge
  pre-scaled by 1/deg_global(post) (K1 with per-edge weights); one reduce-scatter gives each rank
  the exact mean of its post slice, the post projection (K3) runs on that slice only, and one
  all-gather rebuilds the full post table for the next layer and the loss.  A reduce-scatter +
  all-gather moves what one all-reduce does, and the post-side compute is divided by the world
  size instead of replicated;
* post -> post relations (cfg5): edges into the owned post slice, read the full post table;
* backward: every collective's adjoint (all-gather <-> reduce-scatter, all-to-all reversed);
  parameter gradients are summed with one flat all-reduce;
* the link loss is sharded the same way: rank r scores the positive edges of its users against
  the gathered post table; normalised by the GLOBAL edge count and mean(pos_weights), the
  per-rank losses add up to the reference loss (``train_gnn.py:259-281``).

All collectives are asynchronous: the forward ones overlap the local gathers of the same (or
next) layer; gradient exchanges are handed on unfinished (``ops.defer_until``) to their single
consumer so the backward kernels autograd runs in between overlap them.  The compute ops are
injected (``HipImpl`` here; the CPU gloo tests inject plain-torch ops to check the partitioning
logic).
"""
from __future__ import annotations

import dataclasses
import os
import time
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from . import ops
from .graph import RelationCSR, relation_csr
from .nn import HeteroSAGE, Layout, _fused_weights, _LayoutModel
from .synth import ENGAGES, REV_ENGAGES

EdgeType = Tuple[str, str, str]

RELATIONS = [(REV_ENGAGES, 1.0), (ENGAGES, 1.0)]


class CollectiveTrace:
    """Per-collective timing of the sharded step (bench.py's per-kernel timer run at N > 1,
    VERDICT r5 #2): a mark on the issuing stream when a collective is issued, and on the
    consumer's stream just before and just after the consumer's ``wait()``.
      * issue -> after: the collective's latency as its consumer sees it (cover + stall);
      * before -> after: the stall it caused (the consumer's stream waited that long for it);
      * issue -> before: the compute issued under it (its cover).
    With RCCL the marks are HIP events (``wait()`` is a stream wait, no host sync); on the CPU
    (the gloo rehearsal) host clock readings.  ``begin_step()`` starts a step's list, so the
    collectives line up by their position in the step across steps and ranks."""

    def __init__(self, device: torch.device):
        self.cuda = device.type == "cuda"
        self.steps: List[List[dict]] = []

    def begin_step(self):
        self.steps.append([])

    def _mark(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def issue(self, op: str, nbytes: int) -> dict:
        if not self.steps:
            self.begin_step()
        rec = {"op": op, "bytes": int(nbytes), "issue": self._mark()}
        self.steps[-1].append(rec)
        return rec

    def before_wait(self, rec: dict):
        if "pre" not in rec:
            rec["pre"] = self._mark()

    def after_wait(self, rec: dict):
        if "post" not in rec:
            rec["post"] = self._mark()

    def _ms(self, a, b) -> float:
        return float(a.elapsed_time(b)) if self.cuda else (b - a) * 1e3

    def per_position(self) -> List[dict]:
        """Means over the recorded steps, per collective position: op, bytes, wait_ms (issue ->
        after), stall_ms (before -> after), cover_ms (issue -> before).  Call after a device
        synchronise.  A position some step did not wait for is left out of that step's mean."""
        if not self.steps:
            return []
        M = min(len(st) for st in self.steps)
        out = []
        for j in range(M):
            recs = [st[j] for st in self.steps if "pre" in st[j] and "post" in st[j]]
            r0 = self.steps[0][j]
            row = {"op": r0["op"], "bytes": r0["bytes"], "n": len(recs)}
            if recs:
                row["wait_ms"] = sum(self._ms(r["issue"], r["post"]) for r in recs) / len(recs)
                row["stall_ms"] = sum(max(0.0, self._ms(r["pre"], r["post"]))
                                      for r in recs) / len(recs)
                row["cover_ms"] = sum(self._ms(r["issue"], r["pre"]) for r in recs) / len(recs)
            out.append(row)
        return out


_TRACE: Optional[CollectiveTrace] = None


def set_collective_trace(trace: Optional[CollectiveTrace]) -> None:
    """Record every collective DistEnv issues into ``trace`` (None: stop)."""
    global _TRACE
    _TRACE = trace


def _issue(op: str, t: torch.Tensor):
    return _TRACE.issue(op, t.numel() * t.element_size()) if _TRACE is not None else None


def _sync_done(rec):
    """A collective that completed in its call (gloo over device tensors, the blocking all-reduce):
    the consumer waited from the issue on (no cover), until the mark taken after the call (with
    RCCL recorded behind the stream wait the call enqueued)."""
    if rec is not None and _TRACE is not None:
        rec.setdefault("pre", rec["issue"])
        _TRACE.after_wait(rec)


@dataclasses.dataclass
class DistEnv:
    world: int = 1
    rank: int = 0
    group: Optional[object] = None
    # backward all-gather adjoints finish on a side stream and are handed on unfinished (see
    # _AllGather); None = with RCCL only.  Tests set True to run that path over gloo.
    side_adjoint: Optional[bool] = None

    def use_side_adjoint(self, t: torch.Tensor) -> bool:
        if self.side_adjoint is not None:
            return self.side_adjoint and t.is_cuda
        return t.is_cuda and dist.get_backend(self.group) == "nccl"

    @classmethod
    def from_torch(cls) -> "DistEnv":
        if dist.is_available() and dist.is_initialized():
            return cls(dist.get_world_size(), dist.get_rank())
        return cls()

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            rec = _issue("all_reduce", t)
            dist.all_reduce(t, group=self.group)
            _sync_done(rec)
        return t

    def post_slice(self, n: int) -> Tuple[int, int, int]:
        """(slice rows, lo, hi): rank r owns rows [r*S, r*S+S) of the table padded to world*S."""
        S = -(-n // self.world) if n else 0
        return S, self.rank * S, self.rank * S + S

    def _direct(self, t: torch.Tensor) -> bool:
        """RCCL, or gloo on host tensors (the CPU tests), run the tensor collectives as is; gloo
        on device tensors (a one-GPU rehearsal) goes through all-reduce / all_gather lists."""
        return dist.get_backend(self.group) == "nccl" or not t.is_cuda

    def reduce_scatter_async(self, full: torch.Tensor, out: Optional[torch.Tensor] = None):
        """Sum over ranks of ``full`` [world*S, ...]; returns (this rank's slice [S, ...], work).
        ``out``: a contiguous [S, ...] buffer (e.g. a row range of a larger table) to land in."""
        S = full.shape[0] // self.world
        if out is None:
            out = torch.empty((S,) + tuple(full.shape[1:]), dtype=full.dtype, device=full.device)
        rec = _issue("reduce_scatter", full)
        if self._direct(full):
            work = dist.reduce_scatter_tensor(out, full, group=self.group, async_op=True)
            return out, _Held(work, full, out, rec=rec)
        t = full.clone()
        dist.all_reduce(t, group=self.group)
        out.copy_(t[self.rank * S:(self.rank + 1) * S])
        _sync_done(rec)
        return out, _Done()

    def all_gather_async(self, own: torch.Tensor):
        """Concatenation over ranks of ``own`` [S, ...]; returns (full [world*S, ...], work)."""
        full = torch.empty((own.shape[0] * self.world,) + tuple(own.shape[1:]), dtype=own.dtype,
                           device=own.device)
        rec = _issue("all_gather", full)
        if self._direct(own):
            work = dist.all_gather_into_tensor(full, own, group=self.group, async_op=True)
            return full, _Held(work, own, full, rec=rec)
        dist.all_gather(list(full.chunk(self.world)), own, group=self.group)
        _sync_done(rec)
        return full, _Done()

    def broadcast_slices_async(self, own: torch.Tensor):
        """The all-gather of ``own`` [S, ...] as one broadcast per source rank, each straight
        into its row block of the full table (no copy back); returns (full [world*S, ...],
        [work per source rank]).  A consumer that needs only some row blocks waits for those
        (the loss's dP gather runs block by block as they land).  Every rank issues the
        broadcasts in source-rank order."""
        S = own.shape[0]
        full = torch.empty((S * self.world,) + tuple(own.shape[1:]), dtype=own.dtype,
                           device=own.device)
        if not self._direct(own):
            rec = _issue("all_gather", full)
            dist.all_gather(list(full.chunk(self.world)), own, group=self.group)
            _sync_done(rec)
            return full, [_Done() for _ in range(self.world)]
        full[self.rank * S:(self.rank + 1) * S].copy_(own)
        works = []
        for q in range(self.world):
            blk = full[q * S:(q + 1) * S]
            rec = _issue(f"broadcast[src={q}]", blk)
            w = dist.broadcast(blk, src=q, group=self.group, async_op=True)
            works.append(_Done() if q == self.rank and w is None else
                         _Held(w, own, full, rec=rec))
        return full, works

    def all_to_all_async(self, inp: torch.Tensor, send_splits, recv_splits):
        """Rows ``inp[sum(send_splits[:q]) : ...]`` go to rank q; returns (received rows, in rank
        order, work).  Split lists are host ints (static per graph: no size exchange per call)."""
        out = inp.new_empty((int(sum(recv_splits)),) + tuple(inp.shape[1:]))
        rec = _issue("all_to_all", inp)
        if self._direct(inp):
            work = dist.all_to_all_single(out, inp, list(recv_splits), list(send_splits),
                                          group=self.group, async_op=True)
            return out, _Held(work, inp, out, rec=rec)
        # gloo over device tensors (one-GPU rehearsal): the exchange goes through host memory
        host = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(host, inp.cpu(), list(recv_splits), list(send_splits),
                               group=self.group)
        out.copy_(host)
        _sync_done(rec)
        return out, _Done()

    def all_reduce_async(self, t: torch.Tensor):
        """Start an in-place all-reduce; ``.wait()`` on the result before reading ``t`` (with
        NCCL/RCCL that is a stream wait, so kernels enqueued in between overlap the collective)."""
        if self.world > 1:
            rec = _issue("all_reduce", t)
            return _Held(dist.all_reduce(t, group=self.group, async_op=True), t, rec=rec)
        return _Done()


class _Done:
    def wait(self):
        return True


class _Held:
    """An async collective's Work plus references to its buffers until ``wait()`` (gloo's async
    ops do not keep a temporary input alive on their own)."""

    def __init__(self, work, *refs, rec: Optional[dict] = None):
        self.work, self.refs = work, refs
        self.rec, self.trace = rec, _TRACE if rec is not None else None

    def wait(self):
        if self.trace is not None:
            self.trace.before_wait(self.rec)
        # gloo finishes an async collective by copying into the output at wait(); outside no_grad
        # autograd would record that copy on an output it already tracks and cut its graph
        with torch.no_grad():
            self.work.wait()
        if self.trace is not None:
            self.trace.after_wait(self.rec)
        self.refs = None
        return True


class _AllOf:
    """Waits for every handle in a list (the per-source broadcasts of the post table)."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        return True


# The last forward gather of the post table (the loss's input) as per-source broadcasts whose
# row blocks the loss's dP gather consumes as they land (DistEnv.broadcast_slices_async): the own
# block first, then the others in landing order in groups of HGNN_CHUNK_GROUP (2) blocks.  The
# broadcasts land one by one (one link: ~0.42 ms per 64 MB block at N = 8) and the dP gather of a
# block takes ~0.49 ms, so groups of two keep the gather just behind the link.  (Measured and
# not kept, DESIGN.md §7: one all-gather and one dP launch; one launch per block; own block /
# blocks below / blocks above, whose "blocks above" waited for all seven broadcasts — rank 0
# stalled 2.3 ms on the one-link replay, round 4.)
CHUNK_GROUP = int(os.environ.get("HGNN_CHUNK_GROUP", "2"))
# the first group's size: the own block's dP gather (~0.66 ms at N = 8) covers one landed block,
# not two (HGNN_CHUNK_FIRST)
CHUNK_FIRST = int(os.environ.get("HGNN_CHUNK_FIRST", "1"))

# user->post partial sums at world > 1 in this many row ranges of every slice (1 = one
# reduce-scatter of the whole padded table, round 3).  With 2, the first range's reduce-scatter
# is issued after half the gather and the second after the rest, so the link starts while the
# gather runs; the backward's all-gather of the slice gradients is split the same way and its K2
# starts on the first range while the second lands.  HGNN_SPLIT_PARTIALS=1|2.
SPLIT_PARTIALS = int(os.environ.get("HGNN_SPLIT_PARTIALS", "2"))


class Pending:
    """Handle of an in-flight forward all-reduce (see ``all_reduce_sum``)."""
    work = None

    def wait(self):
        if self.work is not None:
            with torch.no_grad():
                self.work.wait()
            self.work = None


class _AllReduceSum(torch.autograd.Function):
    """y = sum over ranks of x (replicated result); adjoint: the same all-reduce of gradients.

    Both directions are issued asynchronously.  Forward: the caller gets ``handle`` and waits on
    it right before consuming y, after enqueueing independent work.  Backward (``defer_grad``):
    the gradient is handed on with the collective still in flight, registered with
    ``ops.defer_until``; its consumer (``ops.weighted_gather``'s backward) waits on it, so the
    autograd nodes that run in between — the user-side backward — overlap it."""

    @staticmethod
    def forward(ctx, x, env: DistEnv, handle: "Pending", defer_grad: bool):
        ctx.env, ctx.defer = env, defer_grad
        y = x.contiguous().clone()
        handle.work = env.all_reduce_async(y)
        return y

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        work = ctx.env.all_reduce_async(g)
        if ctx.defer and ctx.env.world > 1:
            ops.defer_until(g, work)
        else:
            work.wait()
        return g, None, None, None


def all_reduce_sum(x: torch.Tensor, env: DistEnv, handle: Optional[Pending] = None,
                   defer_grad: bool = False) -> torch.Tensor:
    """Sum over ranks.  Without ``handle`` the result is ready on return; with one, call
    ``handle.wait()`` before using it."""
    own = handle is None
    handle = handle or Pending()
    y = _AllReduceSum.apply(x, env, handle, defer_grad)
    if own:
        handle.wait()
    return y


class _ReduceScatter(torch.autograd.Function):
    """This rank's slice of the sum over ranks; adjoint: all-gather of the slice gradients
    (issued asynchronously and, with ``defer_grad``, awaited by its single consumer)."""

    @staticmethod
    def forward(ctx, full, env: DistEnv, handle: "Pending", defer_grad: bool):
        ctx.env, ctx.defer = env, defer_grad
        out, handle.work = env.reduce_scatter_async(full.contiguous())
        return out

    @staticmethod
    def backward(ctx, g):
        full, work = ctx.env.all_gather_async(g.contiguous())
        if ctx.defer:
            ops.defer_until(full, work)
        else:
            work.wait()
        return full, None, None, None


class _EventWait:
    """A deferred gradient's completion as a recorded stream event (``ops.defer_until``)."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True


_SIDE: Dict[torch.device, torch.cuda.Stream] = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(dev)
    return s


class _AllGather(torch.autograd.Function):
    """Concatenation of every rank's slice; adjoint: reduce-scatter of the gradient.

    With ``keep`` the slice is also returned as a second output (a copy) for the next layer's
    root term, so the slice's two gradients — the reduce-scatter and the root's — meet inside
    this backward rather than in autograd's accumulation, which would need the reduce-scatter
    finished on the main stream.  Over RCCL (``defer``) the wait for the reduce-scatter and the
    add run on a side stream, and the result is handed on unfinished to its single consumer
    (the slice projection's backward, via ``ops.defer_until``): the main stream goes on with
    the user-side backward while the collective runs."""

    @staticmethod
    def forward(ctx, own, env: DistEnv, handle: "Pending", keep: bool, defer: bool):
        ctx.env, ctx.defer = env, defer
        full, handle.work = env.all_gather_async(own.contiguous())
        if keep:
            return full, own.clone()
        return full

    @staticmethod
    def backward(ctx, g, g_own=None):
        out, work = ctx.env.reduce_scatter_async(g.contiguous())
        if not (ctx.defer and ctx.env.use_side_adjoint(out)):
            work.wait()
            if g_own is not None:
                out = out + g_own
            return out, None, None, None, None
        main = torch.cuda.current_stream(out.device)
        side = _side_stream(out.device)
        side.wait_stream(main)                # g_own (and the collective's input) are ready
        with torch.cuda.stream(side):
            work.wait()                       # the side stream waits for the reduce-scatter
            if g_own is not None:
                out.add_(g_own)
            ev = torch.cuda.Event()
            ev.record(side)
        out.record_stream(side)
        if g_own is not None:
            g_own.record_stream(side)
        ops.defer_until(out, _EventWait(ev))
        return out, None, None, None, None


class _AllToAll(torch.autograd.Function):
    """Halo exchange: rows to each peer -> rows from each peer; adjoint: the reverse exchange of
    the gradients (issued asynchronously; with ``defer_grad`` awaited by its single consumer, the
    backward of the gather that picked the sent rows)."""

    @staticmethod
    def forward(ctx, x, env: DistEnv, send_splits, recv_splits, handle: "Pending",
                defer_grad: bool):
        ctx.env, ctx.splits, ctx.defer = env, (send_splits, recv_splits), defer_grad
        out, handle.work = env.all_to_all_async(x.contiguous(), send_splits, recv_splits)
        return out

    @staticmethod
    def backward(ctx, g):
        send_splits, recv_splits = ctx.splits
        gx, work = ctx.env.all_to_all_async(g.contiguous(), recv_splits, send_splits)
        if ctx.defer:
            ops.defer_until(gx, work)
        else:
            work.wait()
        return gx, None, None, None, None, None


def user_range(n_users: int, world: int, rank: int) -> Tuple[int, int]:
    m = -(-n_users // world)
    lo = min(n_users, rank * m)
    return lo, min(n_users, lo + m)


def shard_edge_filter(n_users: int, n_posts: int, world: int, rank: int,
                      slice_inputs: bool = False):
    """``keep(edge_type, src, dst) -> bool mask``: the edges rank ``rank`` of ``UserShard`` reads
    (``synth.make_graph(keep=...)`` generates only those): edges into its users (post -> user,
    user -> user), out of its users (user -> post; with ``slice_inputs`` also every edge into its
    post slice), into its post slice (post -> post).  UserShard's own selection from these is the
    one it makes from the global edges, in the same order, so the step is the same bit for bit
    (tests/test_distributed.py)."""
    lo, hi = user_range(n_users, world, rank)
    S = -(-n_posts // world) if n_posts else 0
    p_lo, p_hi = rank * S, rank * S + S

    def keep(et, src, dst):
        if (et[0], et[2]) == ("user", "post"):
            m = (src >= lo) & (src < hi)
            if slice_inputs:
                m |= (dst >= p_lo) & (dst < p_hi)
            return m
        if et[2] == "user":
            return (dst >= lo) & (dst < hi)
        return (dst >= p_lo) & (dst < p_hi)
    return keep


class HipImpl:
    """The MI355X kernels behind the partitioned step."""

    # weighted_gather's backward awaits a gradient whose all-reduce is still in flight
    defer_grad = True
    # linear_fwd_raw / linear_bwd_raw take the ReLU mask in bit form (mask_out= / mask=)
    relu_masks = True
    # the fused weight of a destination update and its adjoint: one launch each
    fused_weights = staticmethod(_fused_weights)

    @staticmethod
    def grads_to_params(convs, msgs, dW, db):
        _grads_to_params(convs, msgs, dW, db)

    def relation(self, edge_index, n_src, n_dst):
        return relation_csr(edge_index, n_src, n_dst)   # cached: the loss finds the same one

    def edge_weights_fwd(self, rel: RelationCSR, w_dst: torch.Tensor) -> torch.Tensor:
        """w_dst[destination] per forward-CSR position (rows are destinations)."""
        counts = (rel.fwd.rowptr[1:] - rel.fwd.rowptr[:-1]).long()
        return torch.repeat_interleave(w_dst, counts).contiguous()

    def edge_weights_bwd(self, rel: RelationCSR, w_dst: torch.Tensor) -> torch.Tensor:
        """w_dst[destination] per CSC position (col holds the destination)."""
        return w_dst[rel.bwd.col.long()].contiguous()

    mean_gather = staticmethod(ops.mean_gather)
    weighted_gather = staticmethod(ops.weighted_gather)
    fused_linear = staticmethod(ops.fused_linear)

    @staticmethod
    def edge_bce_loss(U, P, pos, neg, n_total, cscale, neg_order="edge", ready=None):
        return ops.edge_bce_loss(U, P, pos, neg, None, neg_order=neg_order, check=False,
                                 n_edges_total=n_total, cscale=cscale, ready=ready)

    # raw kernels (no autograd) for UserShard.step's explicit schedule
    gather_mean_raw = staticmethod(ops.gather_mean)
    weighted_gather_raw = staticmethod(ops.weighted_gather_raw)
    weighted_scatter_bwd_raw = staticmethod(ops.weighted_scatter_bwd_raw)
    linear_fwd_raw = staticmethod(ops.linear_fwd)
    linear_bwd_raw = staticmethod(ops.linear_bwd)
    edge_bce_loss_raw = staticmethod(ops.edge_bce_loss_raw)
    presort_negatives = staticmethod(ops.presort_negatives)

    @staticmethod
    def scatter_mean_bwd_raw(g, rel, out=None):
        return ops.scatter_mean_bwd(g, rel, out=out)


def _grads_to_params(convs, msgs, dW: torch.Tensor, db: Optional[torch.Tensor]) -> None:
    """Adjoint of ``nn._fused_weights``: W = [w_1 W_l,1 | ... | w_R W_l,R | sum_r w_r W_r,r],
    b = sum_r w_r b_r, split back into every parameter's gradient by one launch
    (``ops.split_weight_grads``) and accumulated into its ``.grad``."""
    ks, scales, dwl, dwr, dbl = [], [], [], [], []
    for name, _, wt in msgs:
        conv = convs[name]
        ks.append(int(conv.lin_l.weight.shape[1]))
        scales.append(wt)
        dwl.append(torch.empty_like(conv.lin_l.weight))
        dwr.append(torch.empty_like(conv.lin_r.weight) if conv.lin_r is not None else None)
        dbl.append(torch.empty_like(conv.lin_l.bias)
                   if conv.lin_l.bias is not None and db is not None else None)
    k_root = int(dW.shape[1]) - sum(ks)
    ops.split_weight_grads(dW, db, ks, k_root, scales, dwl, dwr, dbl)
    for (name, _, _), gl, gr, gb in zip(msgs, dwl, dwr, dbl):
        conv = convs[name]
        for p, g in ((conv.lin_l.weight, gl), (conv.lin_r.weight if conv.lin_r is not None
                                                 else None, gr), (conv.lin_l.bias, gb)):
            if p is None or g is None:
                continue
            if p.grad is None:
                p.grad = g
            else:
                p.grad.add_(g)


def model_layers(model) -> List[Tuple[Dict[str, torch.nn.Module], Layout]]:
    """[(convs, layout)] per layer: ``HeteroSAGE`` (relation list, L layers) or a
    ``WeightedRGCN``-style layout model (one layer, ``train_gnn.py:155-200``)."""
    if isinstance(model, HeteroSAGE):
        layout: Layout = {}
        for et, w in model.relations:
            layout.setdefault(et[2], []).append(("__".join(et), et, w))
        return [(convs, layout) for convs in model.layers]
    if isinstance(model, _LayoutModel):
        lay = model.layout
        return [({n: getattr(model, n) for msgs in lay.values() for n, _, _ in msgs}, lay)]
    raise TypeError(f"no partitioned forward for {type(model).__name__}")


@dataclasses.dataclass
class _Rel:
    """One relation's share on this rank: its kind ((src type, dst type)), local CSR and (for
    user->post partial sums) the per-position 1/deg_global weights."""
    kind: Tuple[str, str]
    csr: object
    w_fwd: Optional[torch.Tensor] = None
    w_bwd: Optional[torch.Tensor] = None
    # user->post: the same 1/deg_global per destination row (w_fwd is it per position), for the
    # source-blocked form of the partial-sum gather over a multi-GB user table
    row_w: Optional[torch.Tensor] = None
    # user->post only, with ``UserShard(slice_inputs=True)``: every edge INTO the owned post slice
    # (global user ids).  Layer 1 reads the static input user table, which each rank can hold
    # whole: the slice's mean is then computed locally, with no partial sums to reduce-scatter.
    slice_csr: object = None
    # world > 1: the same edges split by the row range of every post slice their post lies in
    # (_PartialHalf).  user->post: the partial sums travel as one reduce-scatter per range, the
    # first issued while the second range's gather still runs; post->user: the K2 of a
    # pre-projected relation's dz into the post table, one reduce-scatter per range likewise
    # (see SPLIT_PARTIALS)
    halves: Optional[List["_PartialHalf"]] = None


@dataclasses.dataclass
class _PartialHalf:
    """A relation's edges whose post lies in rows [lo, hi) of its owner's slice, the post ids
    renumbered into a table of world * (hi - lo) rows in which owner q's rows come q-th: a
    reduce-scatter of such a table hands every rank rows [lo, hi) of its own slice, and an
    all-gather of those rows builds it.  user->post: w_fwd / row_w the partial sums' 1/deg(post)
    and w_bwd its adjoint; post->user: w_bwd = 1/deg(user) per edge, the mean's K2 over the
    whole relation's degrees."""
    csr: object
    w_fwd: Optional[torch.Tensor]
    w_bwd: torch.Tensor
    row_w: Optional[torch.Tensor]
    lo: int
    hi: int


@dataclasses.dataclass
class _Halo:
    """Remote source users of this rank's user->user edges.  ``rel_send`` picks the owned rows
    every peer asked for (grouped by peer; a K1 gather of degree-1 rows whose K2 adjoint sums the
    returned gradients per row, deterministically); received rows follow in rank order, so halo
    row k is ``remote[k]``."""
    rel_send: object
    send_splits: List[int]
    recv_splits: List[int]
    n_halo: int


class UserShard:
    """Static per-rank structures of a destination-partitioned user<->post graph.

    ``edges``: the global ``edge_index_dict`` (any of ``post->user``, ``user->user``,
    ``user->post``, ``post->post`` relations; ``engages`` is also the loss's positive edges) or,
    for the two-relation training graph, the global ``engages`` tensor alone (its flip is the
    ``rev_engages`` relation, ``train_gnn.py:142``).  Rank r owns users [lo, hi) and post rows
    [p_lo, p_hi) of the table padded to world * S rows:

    * post->user  (rev_engages, followed_by): edges into owned users; sources from the full
      (all-gathered) post table — complete locally;
    * user->user  (social): edges into owned users; remote sources arrive by one all-to-all
      halo exchange per layer (the rows each peer asked for at setup), gradients return by the
      reverse exchange;
    * user->post  (engages): edges out of owned users, each pre-scaled by 1/deg_global(post);
      partial sums over the padded table, one reduce-scatter per relation gives the exact
      mean of the owned slice;
    * post->post: edges into owned post rows, sources from the full post table.

    ``edges`` may also hold only this rank's share (``shard_edge_filter``) with the global
    positive-edge count as ``num_edges_global``; ``pos_weights`` are then the shard edges'.
    """

    def __init__(self, edges, n_users: int, n_posts: int, env: DistEnv, impl=None,
                 pos_weights: Optional[torch.Tensor] = None, slice_inputs: bool = False,
                 num_edges_global: Optional[int] = None):
        impl = impl or HipImpl()
        self.env, self.impl = env, impl
        self.slice_inputs = slice_inputs
        if torch.is_tensor(edges):
            edges = {ENGAGES: edges, REV_ENGAGES: edges.flip(0)}
        self.n_users, self.n_posts = n_users, n_posts
        self.lo, self.hi = user_range(n_users, env.world, env.rank)
        self.n_own = self.hi - self.lo
        # post table padded to world * S rows; rank r owns rows [r*S, r*S+S)
        self.post_rows, self.p_lo, self.p_hi = env.post_slice(n_posts)
        self.n_posts_pad = self.post_rows * env.world
        n_of = {"user": n_users, "post": n_posts}
        for et, ei in edges.items():
            if et[0] not in n_of or et[2] not in n_of:
                raise ValueError(f"relation {et}: node types must be 'user' / 'post'")
        # the loss's positive edges: engages out of owned users (same tensor as the relation's
        # local edges, so the loss finds the cached CSR)
        self.mask = None
        self.pos_local = None
        self.num_edges_global = 0
        self.rels: Dict[EdgeType, _Rel] = {}
        uu = [et for et in edges if (et[0], et[2]) == ("user", "user")]
        remote = None
        if uu:
            src_all = torch.cat([edges[et][0][self._owned_users(edges[et][1])] for et in uu])
            remote = torch.unique(src_all[~self._owned_users(src_all)])   # sorted
        self.halo = self._setup_halo(remote) if remote is not None else None
        for et, ei in edges.items():
            self.rels[et] = self._local_relation(et, ei, remote)
        if ENGAGES in edges:
            # (edges may be this rank's shard only — shard_edge_filter — with the global count
            # given; the loss is normalised by it)
            self.num_edges_global = (int(num_edges_global) if num_edges_global is not None
                                     else int(edges[ENGAGES].shape[1]))
        self.cscale = None
        if pos_weights is not None:   # global mean of the interaction weights (static)
            if self.mask is None:
                raise ValueError("pos_weights given but the graph has no engages relation")
            s = torch.stack([pos_weights[self.mask].to(torch.float64).sum(),
                             torch.tensor(float(self.mask.sum()), dtype=torch.float64,
                                          device=pos_weights.device)])
            env.all_reduce_(s)
            self.cscale = (s[0] / s[1]).to(torch.float32)

    # ------------------------------------------------------------------ setup
    def _owned_users(self, ids: torch.Tensor) -> torch.Tensor:
        return (ids >= self.lo) & (ids < self.hi)

    def _local_relation(self, et, ei: torch.Tensor, remote) -> _Rel:
        impl, kind = self.impl, (et[0], et[2])
        src, dst = ei[0], ei[1]
        if kind == ("post", "user"):
            m = self._owned_users(dst)
            local = torch.stack([src[m], dst[m] - self.lo]).contiguous()
            return _Rel(kind, impl.relation(local, self.n_posts_pad, self.n_own),
                        halves=self._k2_halves(local))
        if kind == ("user", "user"):
            m = self._owned_users(dst)
            s = src[m]
            own = self._owned_users(s)
            if remote is not None and remote.numel():
                pos = torch.searchsorted(remote, s).clamp_(max=remote.numel() - 1)
                ext = torch.where(own, s - self.lo, self.n_own + pos)
            else:
                ext = s - self.lo
            local = torch.stack([ext, dst[m] - self.lo]).contiguous()
            n_halo = self.halo.n_halo if self.halo is not None else 0
            return _Rel(kind, impl.relation(local, self.n_own + n_halo, self.n_own))
        if kind == ("user", "post"):
            m = self._owned_users(src)
            local = torch.stack([src[m] - self.lo, dst[m]]).contiguous()
            deg = torch.bincount(local[1], minlength=self.n_posts_pad).to(torch.float32)
            self.env.all_reduce_(deg)
            inv = torch.where(deg > 0, 1.0 / deg.clamp(min=1.0), torch.zeros_like(deg))
            rel = impl.relation(local, self.n_own, self.n_posts_pad)
            if et == ENGAGES:
                self.mask, self.pos_local = m, local
            slice_rel = None
            if self.slice_inputs:
                ms = (dst >= self.p_lo) & (dst < self.p_hi)
                sl = torch.stack([src[ms], dst[ms] - self.p_lo]).contiguous()
                slice_rel = impl.relation(sl, self.n_users, self.post_rows)
            return _Rel(kind, rel, impl.edge_weights_fwd(rel, inv), impl.edge_weights_bwd(rel, inv),
                        inv, slice_rel, self._partial_halves(local, inv))
        # post -> post: edges into the owned slice of the post table
        m = (dst >= self.p_lo) & (dst < self.p_hi)
        local = torch.stack([src[m], dst[m] - self.p_lo]).contiguous()
        return _Rel(kind, impl.relation(local, self.n_posts_pad, self.post_rows))

    def _ranges(self):
        """The SPLIT_PARTIALS row ranges of a post slice, or None (world 1, slices too short)."""
        W, S = self.env.world, self.post_rows
        n = min(max(SPLIT_PARTIALS, 1), S)
        if W == 1 or n < 2:
            return None
        return [(S * i // n, S * (i + 1) // n) for i in range(n)]

    def _renumber(self, post: torch.Tensor, lo: int, hi: int):
        """Mask of the padded post ids in rows [lo, hi) of their slice, and their ids in the
        range table (owner q's rows q-th)."""
        S = self.post_rows
        q, j = torch.div(post, S, rounding_mode="floor"), post % S
        m = (j >= lo) & (j < hi)
        return m, q[m] * (hi - lo) + (j[m] - lo)

    def _partial_halves(self, local: torch.Tensor, inv: torch.Tensor):
        """The user->post edges (local user, padded post) per row range (_PartialHalf)."""
        ranges = self._ranges()
        if ranges is None:
            return None
        W, inv_q = self.env.world, inv.view(self.env.world, self.post_rows)
        out = []
        for lo, hi in ranges:
            m, ids = self._renumber(local[1], lo, hi)
            rel = self.impl.relation(torch.stack([local[0][m], ids]).contiguous(), self.n_own,
                                     W * (hi - lo))
            inv_h = inv_q[:, lo:hi].reshape(-1).contiguous()
            out.append(_PartialHalf(rel, self.impl.edge_weights_fwd(rel, inv_h),
                                    self.impl.edge_weights_bwd(rel, inv_h), inv_h, lo, hi))
        return out

    def _k2_halves(self, local: torch.Tensor):
        """The post->user edges (padded post, local user) per row range, each edge weighted by
        1/deg(user) over the whole relation (_PartialHalf)."""
        ranges = self._ranges()
        if ranges is None:
            return None
        deg = torch.bincount(local[1], minlength=self.n_own).to(torch.float32)
        inv_u = 1.0 / deg.clamp(min=1.0)
        out = []
        for lo, hi in ranges:
            m, ids = self._renumber(local[0], lo, hi)
            rel = self.impl.relation(torch.stack([ids, local[1][m]]).contiguous(),
                                     self.env.world * (hi - lo), self.n_own)
            out.append(_PartialHalf(rel, None, self.impl.edge_weights_bwd(rel, inv_u), None,
                                    lo, hi))
        return out

    def _setup_halo(self, remote: torch.Tensor) -> _Halo:
        """Tell every owner which of its rows this rank needs (two all-to-alls, once)."""
        env, world = self.env, self.env.world
        m = -(-self.n_users // world)
        owner = torch.div(remote, m, rounding_mode="floor")
        recv = torch.bincount(owner, minlength=world).to(torch.int64)
        ones = [1] * world
        send, work = env.all_to_all_async(recv, ones, ones)
        work.wait()
        recv_splits, send_splits = recv.tolist(), send.tolist()
        ids, work = env.all_to_all_async(remote.contiguous(), recv_splits, send_splits)
        work.wait()
        n_send = int(sum(send_splits))
        dev = remote.device
        pick = torch.stack([ids - self.lo, torch.arange(n_send, dtype=torch.int64, device=dev)])
        rel_send = self.impl.relation(pick.contiguous(), self.n_own, n_send)
        return _Halo(rel_send, send_splits, recv_splits, int(sum(recv_splits)))

    def local_edges_of(self, per_edge: torch.Tensor) -> torch.Tensor:
        """Slice a per-global-edge tensor (e.g. injected negatives) to this rank's edges."""
        return per_edge[self.mask]

    # ---------------------------------------------------------------- forward
    def _halo_start(self, h_u: torch.Tensor, defer: bool):
        if self.halo is None or self.env.world == 1:
            return None, Pending()
        hl = self.halo
        x_send = self.impl.mean_gather(h_u, hl.rel_send)
        pend = Pending()
        recv = _AllToAll.apply(x_send, self.env, hl.send_splits, hl.recv_splits, pend, defer)
        return recv, pend

    def forward(self, model, x_user_own: torch.Tensor, x_post: torch.Tensor,
                wait: bool = True, x_user_full: Optional[torch.Tensor] = None):
        """Partitioned forward of ``model`` (``HeteroSAGE`` or a ``WeightedRGCN`` layout);
        returns (owned user embeddings, post embeddings of the whole padded table — rows >=
        n_posts are padding).  ``wait=False`` leaves the last all-gather of the post table in
        flight for :meth:`loss`, which waits on it only after enqueueing the negatives sort.
        ``x_user_full`` (the whole input user table, with ``slice_inputs=True``): layer 1's
        user->post means of the owned post slice are computed locally (no reduce-scatter)."""
        impl, env = self.impl, self.env
        if x_post.shape[0] != self.n_posts_pad:
            x_post = torch.nn.functional.pad(x_post, (0, 0, 0, self.n_posts_pad - x_post.shape[0]))
        h_u, h_p = x_user_own, x_post
        h_p_own = x_post[self.p_lo:self.p_hi]
        gathered = None                       # in-flight all-gather of h_p
        defer = getattr(impl, "defer_grad", False)
        layers = model_layers(model)
        n_layers = len(layers)
        for li, (convs, layout) in enumerate(layers):
            shapes = {"user": h_u, "post": h_p}
            umsgs, pmsgs = layout.get("user", []), layout.get("post", [])
            for _, et, _ in umsgs + pmsgs:
                if et not in self.rels:
                    raise KeyError(f"relation {et} is not in the sharded graph")
            # 1. halo rows out, 2. post partial sums out: both collectives in flight while the
            # local gathers below run
            halo, halo_pend = (self._halo_start(h_u, defer) if any(
                et[0] == "user" for _, et, _ in umsgs) else (None, Pending()))
            a_post = {}
            for _, et, _ in pmsgs:
                r = self.rels[et]
                if r.kind[0] == "user":
                    if li == 0 and x_user_full is not None and r.slice_csr is not None:
                        a_post[et] = (impl.mean_gather(x_user_full, r.slice_csr), Pending())
                        continue
                    s = impl.weighted_gather(h_u, r.csr, r.w_fwd, r.w_bwd)
                    pend = Pending()
                    a_post[et] = ((_ReduceScatter.apply(s, env, pend, defer), pend)
                                  if env.world > 1 else (s, pend))
            if gathered is not None:          # the previous layer's all-gather of h_p
                gathered.wait()
                gathered = None
            h_u_next = h_u
            if umsgs:
                Wu, bu = impl.fused_weights(convs, umsgs, shapes)
                segs, x_ext = [], None
                for _, et, _ in umsgs:
                    r = self.rels[et]
                    if r.kind[0] == "post":
                        segs.append(impl.mean_gather(h_p, r.csr))
                    else:
                        if x_ext is None:
                            halo_pend.wait()
                            x_ext = h_u if halo is None else torch.cat([h_u, halo])
                        segs.append(impl.mean_gather(x_ext, r.csr))
                h_u_next = impl.fused_linear(segs + [h_u], Wu, bu, True)
            if pmsgs:
                Wp, bp = impl.fused_weights(convs, pmsgs, shapes)
                segs = []
                for _, et, _ in pmsgs:
                    r = self.rels[et]
                    if r.kind[0] == "post":
                        segs.append(impl.mean_gather(h_p, r.csr))
                    else:
                        a, pend = a_post[et]
                        pend.wait()
                        segs.append(a)
                # the post projection runs on this rank's slice only
                h_p_own = impl.fused_linear(segs + [h_p_own], Wp, bp, True)
                if env.world == 1:
                    h_p = h_p_own
                else:
                    gathered = Pending()
                    if li + 1 < n_layers:     # the slice is also the next layer's root input
                        h_p, h_p_own = _AllGather.apply(h_p_own, env, gathered, True, defer)
                    else:
                        h_p = _AllGather.apply(h_p_own, env, gathered, False, defer)
            h_u = h_u_next
        self._post_pending = gathered or Pending()
        if wait:
            self._post_pending.wait()
        return h_u, h_p

    def step(self, model, x_user_own: torch.Tensor, x_post: torch.Tensor,
             neg_local: torch.Tensor, neg_order: str = "edge",
             x_user_full: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One training step's forward, loss and backward for this rank, with an explicit
        schedule instead of autograd's: the same kernels, and the parameter gradients
        ``forward`` + ``loss`` + ``backward()`` give (accumulated into ``.grad``); returns the
        rank's loss share (detached).  Autograd runs backward nodes newest first, so a
        collective's consumer ran right after the collective was issued and the main stream
        waited for it; here every collective is issued as soon as its input is complete and
        waited for only by its consumer, with independent work in between:

        * the post-table gradient's reduce-scatter runs under the user-side projection
          backward;
        * the post partial sums' slice-gradient all-gather runs under the K2s into the
          previous layer's post table (and the halo's reverse all-to-all);
        * the previous layer's reduce-scatter runs under the user rows' K2s and the next
          projection backward.
        """
        if self.cscale is None:
            raise ValueError("UserShard built without pos_weights")
        with torch.no_grad():
            return _step(self, model, x_user_own, x_post, neg_local, neg_order, x_user_full)

    def loss(self, h_u_own, h_p, neg_local, neg_order="edge"):
        """This rank's additive share of the reference loss."""
        if self.cscale is None:
            raise ValueError("UserShard built without pos_weights")
        pend = getattr(self, "_post_pending", None) or Pending()
        self._post_pending = None
        return self.impl.edge_bce_loss(h_u_own, h_p, self.pos_local, neg_local,
                                       self.num_edges_global, self.cscale, neg_order=neg_order,
                                       ready=pend.wait)


def _issue_slice_gathers(shard, env, pm, dxp, multi):
    """B4: all-gathers of the slice gradients of every user->post relation's partial sums —
    per row range in the forward's layout (_PartialHalf) — as {relation: [(range, (table,
    work))]} (range None: the whole padded table)."""
    gath = {}
    for j, (_, et, _) in enumerate(pm):
        r = shard.rels[et]
        if r.kind[0] == "user":
            if multi and r.halves:
                gath[et] = [(hf, env.all_gather_async(dxp[j][hf.lo:hf.hi].contiguous()))
                            for hf in r.halves]
            else:
                gath[et] = [(None, env.all_gather_async(dxp[j]) if multi
                             else (dxp[j], _Done()))]
    return gath


def _k2_into(impl, buf, g, csr):
    """K2 of ``g`` over ``csr`` added into ``buf``; the first contribution writes a fresh buffer
    (every row, zero where no edge), so no zero fill of the whole table precedes it."""
    if buf is None:
        return impl.scatter_mean_bwd_raw(g, csr)
    impl.scatter_mean_bwd_raw(g, csr, out=buf)
    return buf


def _pre_rel(shard: "UserShard", layers, li: int) -> Optional[int]:
    """Index (into layer ``li``'s user-side relations) of the post -> user relation whose lin_l
    runs on the post SLICE before the previous layer's all-gather, or None.

    ``W (mean_j x_j) = mean_j (W x_j)`` (``ops.use_pre_projection``): each rank projects its
    S = n_posts / world slice rows (y_p_own W_l^T, S x H), the all-gather carries the projected
    rows instead of y_p, and the user-side update loses its [n_own x d] lin_l block — K = 2d ->
    d for the forward, and the backward's dgrad of that block (the relation's K2 scatters the
    masked dz itself).  The adjoint: the reduce-scatter brings the slice's dP, whose projection
    backward (S rows) gives d y_p_own and the block's weight gradient.  Applies when the
    all-gathered table has no other reader: layer li > 0 (layer 0 reads the static inputs), a
    post side in layers li-1 and li (li's post table is not passed through), exactly one
    post -> user relation and no post -> post relation at layer li.  ``HGNN_PREPROJECT=0``
    turns it off (``ops.PRE_PROJECTION``)."""
    if li == 0 or not ops.PRE_PROJECTION or not getattr(shard.impl, "pre_projection", True):
        return None
    _, prev_layout = layers[li - 1]
    _, layout = layers[li]
    um, pm = layout.get("user", []), layout.get("post", [])
    if not prev_layout.get("post") or not pm:
        return None
    if any(shard.rels[et].kind[0] == "post" for _, et, _ in pm):
        return None
    js = [j for j, (_, et, _) in enumerate(um) if shard.rels[et].kind[0] == "post"]
    return js[0] if len(js) == 1 else None


def _block_cols(um, widths: Dict[str, int]) -> List[Tuple[int, int]]:
    """(offset, width) of each user-side relation's lin_l block in the fused weight
    ``[w_1 W_l,1 | ... | w_R W_l,R | root]`` (``nn._fused_weights``)."""
    cols, o = [], 0
    for _, et, _ in um:
        k = widths[et[0]]
        cols.append((o, k))
        o += k
    return cols


def _without_block(W: torch.Tensor, col: Tuple[int, int]) -> torch.Tensor:
    o, k = col
    return torch.cat([W[:, :o], W[:, o + k:]], dim=1).contiguous()


def _lin_fwd(impl, segs, W, b, add, mask=None):
    kw = {} if add is None else {"add": add}
    if mask is not None:
        kw["mask_out"] = mask
    return impl.linear_fwd_raw(segs, W, b, True, **kw)


def _relu_mask(impl, n, h, like):
    """The bit form of a ReLU output's mask for the backward (HIP kernels only), or None."""
    if not getattr(impl, "relu_masks", False):
        return None
    return ops.relu_mask_for(int(n), int(h), True, like.device)


def _lin_bwd(impl, segs, W, dout, y, dxs, need_b, mask, **kw):
    if mask is not None:
        kw["mask"] = mask
    return impl.linear_bwd_raw(segs, W, dout, y, dxs, True, need_b, **kw)


def _step(shard: "UserShard", model, x_user_own, x_post, neg_local, neg_order, x_user_full=None):
    """UserShard.step: forward, loss and backward with every collective issued as early as its
    input exists and waited as late as its consumer allows (see the method docstring)."""
    impl, env = shard.impl, shard.env
    multi = env.world > 1
    if x_post.shape[0] != shard.n_posts_pad:
        x_post = torch.nn.functional.pad(x_post, (0, 0, 0, shard.n_posts_pad - x_post.shape[0]))
    layers = model_layers(model)
    L = len(layers)
    for convs, _ in layers:
        if any(c.lin_r is None for c in convs.values()):
            raise NotImplementedError("UserShard.step expects SAGEConv(root_weight=True) layers")
    pre = [_pre_rel(shard, layers, li) for li in range(L)]
    fused: Dict[int, tuple] = {}
    presorted = None                            # the loss's negatives, grouped ahead of it

    def weights_of(li, shapes):
        if li not in fused:
            convs, layout = layers[li]
            um, pm = layout.get("user", []), layout.get("post", [])
            fused[li] = (impl.fused_weights(convs, um, shapes) if um else (None, None),
                         impl.fused_weights(convs, pm, shapes) if pm else (None, None))
        return fused[li]

    h_u, h_p, h_p_own = x_user_own, x_post, x_post[shard.p_lo:shard.p_hi]
    ag = None                                   # in-flight all-gather of h_p
    proj = [None] * L                           # layer li's pre-projection: (block, cols)
    saved = []
    for li, (convs, layout) in enumerate(layers):
        um, pm = layout.get("user", []), layout.get("post", [])
        for _, et, _ in um + pm:
            if et not in shard.rels:
                raise KeyError(f"relation {et} is not in the sharded graph")
        # h_p is the projected table when this layer pre-projects (proj[li]); the own slice has
        # the width of the previous post output, which the weight shapes need
        shapes = {"user": h_u, "post": h_p_own}
        (Wu, bu), (Wp, bp) = weights_of(li, shapes)
        jp = pre[li] if proj[li] is not None else None
        col_pre = proj[li][1] if jp is not None else None
        # F1 halo rows out; F2 post partial sums -> reduce-scatter (both in flight from here)
        halo, halo_w = None, _Done()
        if multi and shard.halo is not None and any(et[0] == "user" for _, et, _ in um):
            hl = shard.halo
            halo, halo_w = env.all_to_all_async(impl.gather_mean_raw(h_u, hl.rel_send),
                                                hl.send_splits, hl.recv_splits)
        rs, rs_issued = {}, False
        for _, et, _ in pm:
            r = shard.rels[et]
            if r.kind[0] == "user":
                if li == 0 and x_user_full is not None and r.slice_csr is not None:
                    # static inputs held whole: the owned slice's mean, no partial sums to reduce
                    rs[et] = (impl.gather_mean_raw(x_user_full, r.slice_csr), _Done())
                    continue
                if multi and r.halves:
                    # one reduce-scatter per row range of the slices, each issued as soon as
                    # its range's partial sums are enqueued
                    a = h_u.new_empty(shard.post_rows, h_u.shape[1])
                    works = []
                    for hf in r.halves:
                        part = impl.weighted_gather_raw(h_u, hf.csr, hf.w_fwd, hf.row_w)
                        works.append(env.reduce_scatter_async(part, out=a[hf.lo:hf.hi])[1])
                    rs[et] = (a, _AllOf(works))
                else:
                    part = impl.weighted_gather_raw(h_u, r.csr, r.w_fwd, r.row_w)
                    rs[et] = env.reduce_scatter_async(part) if multi else (part, _Done())
                rs_issued = True
        if (multi and rs_issued and li == L - 1 and presorted is None
                and hasattr(impl, "presort_negatives")):
            # the loss's negatives grouped by post now: they need only the edges and the draws,
            # and the sort adds its ~0.5 ms (N = 8) to the compute under this reduce-scatter,
            # the least covered collective of the forward
            presorted = impl.presort_negatives(int(h_u.shape[0]), shard.n_posts_pad,
                                               shard.pos_local, neg_local, neg_order)
        if ag is not None:                      # F3 the previous layer's post table
            ag.wait()
            ag = None
        Wu_main = _without_block(Wu, col_pre) if jp is not None else Wu
        st = {"x_ext": None, "a_u": [], "add": None, "y_u": h_u, "a_p": [],
              "y_p_own": h_p_own, "y_p": h_p, "m_u": None, "m_p": None, "p_chunks": None}

        def user_gathers():
            # F4 user side (a pre-projected relation's mean of projected rows enters the epilogue)
            for j, (_, et, _) in enumerate(um):
                r = shard.rels[et]
                if j == jp:
                    st["add"] = impl.gather_mean_raw(h_p, r.csr)
                elif r.kind[0] == "post":
                    st["a_u"].append(impl.gather_mean_raw(h_p, r.csr))
                else:
                    if st["x_ext"] is None:
                        halo_w.wait()
                        st["x_ext"] = h_u if halo is None else torch.cat([h_u, halo])
                    st["a_u"].append(impl.gather_mean_raw(st["x_ext"], r.csr))

        def user_projection():
            if um:
                st["m_u"] = _relu_mask(impl, h_u.shape[0], Wu_main.shape[0], h_u)
                st["y_u"] = _lin_fwd(impl, st["a_u"] + [h_u], Wu_main, bu, st["add"], st["m_u"])

        def post_side():
            # F5 post side on the owned slice, then its all-gather (of the next layer's projected
            # rows when that layer pre-projects)
            nonlocal ag
            for _, et, _ in pm:
                r = shard.rels[et]
                if r.kind[0] == "post":
                    st["a_p"].append(impl.gather_mean_raw(h_p, r.csr))
                else:
                    a, w = rs[et]
                    w.wait()
                    st["a_p"].append(a)
            if not pm:
                return
            st["m_p"] = _relu_mask(impl, h_p_own.shape[0], Wp.shape[0], h_p_own)
            y_p_own = _lin_fwd(impl, st["a_p"] + [h_p_own], Wp, bp, None, st["m_p"])
            table = y_p_own
            nxt = li + 1
            if nxt < L and pre[nxt] is not None:
                wu = int(Wu.shape[0]) if um else int(h_u.shape[1])   # the next layer's input widths
                wp = int(y_p_own.shape[1])
                stand_in = {"user": h_u.new_empty((0, wu)), "post": h_u.new_empty((0, wp))}
                (Wu_n, _), _ = weights_of(nxt, stand_in)
                o, k = _block_cols(layers[nxt][1]["user"], {"user": wu, "post": wp})[pre[nxt]]
                if k >= Wu_n.shape[0]:          # the projected rows are no wider than y_p
                    block = Wu_n[:, o:o + k].contiguous()
                    table = impl.linear_fwd_raw([y_p_own], block, None, False)
                    proj[nxt] = (block, (o, k))
            st["y_p_own"] = y_p_own
            if multi and nxt == L:
                # the loss's post table: one broadcast per source rank, so the dP gather can run
                # on each row block as it lands (own block first) instead of after all of them
                st["y_p"], works = env.broadcast_slices_async(table)
                S, r, W = shard.post_rows, env.rank, env.world
                others = [q for q in range(W) if q != r]
                first = max(1, CHUNK_FIRST)
                groups = [others[:first]] + [
                    others[i:i + max(1, CHUNK_GROUP)]
                    for i in range(first, len(others), max(1, CHUNK_GROUP))]
                groups = [grp for grp in groups if grp]
                st["p_chunks"] = [(r * S, (r + 1) * S, None)]
                for grp in groups:
                    # a group of blocks contiguous in rows (the own block splits at most one)
                    runs = []
                    for q in grp:
                        if runs and runs[-1][1] == q * S:
                            runs[-1][1] = (q + 1) * S
                        else:
                            runs.append([q * S, (q + 1) * S])
                    wait = (lambda qs: (lambda: [works[q].wait() for q in qs]))(grp)
                    for k, (lo, hi) in enumerate(runs):
                        st["p_chunks"].append((lo, hi, wait if k == 0 else None))
                ag = _AllOf(works)
            else:
                st["y_p"], ag = env.all_gather_async(table) if multi else (table, None)

        if multi and pm and not rs_issued:
            # no reduce-scatter to wait for (layer 1 with the static inputs held whole): the post
            # side first, so its all-gather runs under this layer's user side and the next
            # layer's partial sums
            post_side()
            user_gathers()
            user_projection()
        else:
            # the loss's dP gather covers the last post table's broadcasts, so the user
            # projection goes first, under the reduce-scatter
            user_gathers()
            user_projection()
            post_side()
        x_ext, a_u, add, y_u = st["x_ext"], st["a_u"], st["add"], st["y_u"]
        p_chunks = st["p_chunks"]
        a_p, y_p_own, y_p = st["a_p"], st["y_p_own"], st["y_p"]
        masks = (st["m_u"], st["m_p"])
        saved.append((convs, um, pm, h_u, h_p, h_p_own, x_ext, a_u, a_p, y_u, y_p_own, Wu_main,
                      Wp, bu is not None, bp is not None, jp, col_pre, masks))
        h_u, h_p, h_p_own = y_u, y_p, y_p_own
    shard.pre_layers = [li for li in range(L) if proj[li] is not None]   # (for tests)
    # loss: the negatives sort runs while the last all-gather lands; dP's reduce-scatter (the
    # all-gather's adjoint, B1) is issued as soon as dP is enqueued and runs under the scoring
    # pass and the user-side projection backward
    R = None                                    # reduce-scatter of G_full, once issued

    def issue_b1(dP):
        nonlocal R
        if multi and layers[-1][1].get("post"):
            R = env.reduce_scatter_async(dP)

    loss, G_u, G_full = impl.edge_bce_loss_raw(h_u, h_p, shard.pos_local, neg_local,
                                               shard.num_edges_global, shard.cscale, neg_order,
                                               ag.wait if ag is not None else None,
                                               on_dP=issue_b1, p_chunks=p_chunks,
                                               **({"presorted": presorted} if presorted is not None
                                                  else {}))
    G_own = None
    R_proj = None                               # (block, cols, grads to finish) if R carries dP
    for li in reversed(range(L)):
        (convs, um, pm, hu, hp, hpo, x_ext, a_u, a_p, yu, ypo, Wu, Wp, has_bu, has_bp, jp,
         col_pre, (m_u, m_p)) = saved[li]
        need_x = li > 0                         # layer 0's inputs are the (fixed) features
        if pm and R is None:                    # B1 adjoint of the post-table all-gather
            g = G_full if G_full is not None else ypo.new_zeros(shard.n_posts_pad, ypo.shape[1])
            R = env.reduce_scatter_async(g) if multi else (g, _Done())
        def b2a():
            # B2a user-side projection backward (a pre-projected relation: dz as a side output)
            dxu, dz, pending_w = [], None, None
            if um:
                dxu = [torch.empty_like(a) if need_x else None for a in a_u]
                dxu.append(torch.empty_like(hu) if need_x else None)
                if jp is not None:
                    dz = torch.empty_like(G_u)
                    dW, db = _lin_bwd(impl, a_u + [hu], Wu, G_u.contiguous(), yu, dxu, has_bu,
                                      m_u, dz_out=dz)
                    pending_w = (convs, um, dW, db, col_pre)  # the block's gradient comes with dP
                else:
                    dW, db = _lin_bwd(impl, a_u + [hu], Wu, G_u.contiguous(), yu, dxu, has_bu,
                                      m_u)
                    impl.grads_to_params(convs, um, dW, db)
                d_hu = dxu[-1]
            else:
                d_hu = G_u if need_x else None
            return dxu, dz, pending_w, d_hu

        def b3():
            # B3 post-side projection backward (waits for the reduce-scatter)
            nonlocal R, R_proj
            dxp, d_hpo = [], G_own
            if pm:
                r_slice, r_w = R
                r_w.wait()
                R = None
                if R_proj is not None:
                    # the reduce-scatter brought the next layer's dP slice: the projection's
                    # backward (S rows) gives this layer's output-slice gradient and the block's
                    block, (o, k), (n_convs, n_um, n_dW, n_db, _) = R_proj
                    R_proj = None
                    g_y = torch.empty_like(ypo)
                    dblock, _ = impl.linear_bwd_raw([ypo], block, r_slice.contiguous(), None,
                                                    [g_y], True, False)
                    dW_full = torch.cat([n_dW[:, :o], dblock, n_dW[:, o:]], dim=1)
                    impl.grads_to_params(n_convs, n_um, dW_full, n_db)
                    r_slice = g_y
                g_slice = r_slice if G_own is None else r_slice + G_own
                dxp = [torch.empty_like(a) if need_x else None for a in a_p]
                dxp.append(torch.empty_like(hpo) if need_x else None)
                dW, db = _lin_bwd(impl, a_p + [hpo], Wp, g_slice.contiguous(), ypo, dxp, has_bp,
                                  m_p)
                impl.grads_to_params(convs, pm, dW, db)
                d_hpo = dxp[-1]
            return dxp, d_hpo

        # The loss's layer: its reduce-scatter (dP) has had the rest of the loss under it, so the
        # post side goes first and its slice gradients' all-gather then runs under the user-side
        # backward as well; lower layers keep the user side first, under their reduce-scatter.
        if li == L - 1 and multi:
            dxp, d_hpo = b3()
            ag_early = _issue_slice_gathers(shard, env, pm, dxp, multi) if need_x else {}
            dxu, dz, pending_w, d_hu = b2a()
        else:
            dxu, dz, pending_w, d_hu = b2a()
            dxp, d_hpo = b3()
            ag_early = None
        if not need_x:
            break
        # B4 slice gradients of the post partial sums: all-gather (in flight over B2b)
        gath = ag_early if ag_early is not None else _issue_slice_gathers(shard, env, pm, dxp,
                                                                          multi)
        # B2b gradients into the previous layer's post table (of its projected rows when this
        # layer pre-projects: the K2 of dz) and the halo (a layer without a post side passes the
        # table through: its gradient flows on unchanged)
        G_prev = None if pm else G_full
        d_xext = None
        ai = 0
        prev_pm = saved[li - 1][2]
        R_split = None                          # the K2 of dz per row range, each reduce-scattered
        for j, (_, et, _) in enumerate(um):
            r = shard.rels[et]
            if j == jp:
                if multi and r.halves and prev_pm and G_prev is None:
                    # (the only contribution to this table: _pre_rel admits no other relation
                    # into it) one reduce-scatter per range, the first under the second's K2
                    g_sl = dz.new_empty(shard.post_rows, dz.shape[1])
                    works = [env.reduce_scatter_async(
                        impl.weighted_scatter_bwd_raw(dz, hf.csr, hf.w_bwd),
                        out=g_sl[hf.lo:hf.hi])[1] for hf in r.halves]
                    R_split = (g_sl, _AllOf(works))
                else:
                    G_prev = _k2_into(impl, G_prev, dz, r.csr)
                continue
            if r.kind[0] == "post":
                G_prev = _k2_into(impl, G_prev, dxu[ai], r.csr)
            else:
                d_xext = _k2_into(impl, d_xext, dxu[ai], r.csr)
            ai += 1
        for j, (_, et, _) in enumerate(pm):
            r = shard.rels[et]
            if r.kind[0] == "post":
                G_prev = _k2_into(impl, G_prev, dxp[j], r.csr)
        back, back_w = None, _Done()
        if d_xext is not None:
            n_own = hu.shape[0]
            d_hu.add_(d_xext[:n_own])
            # every rank joins the reverse exchange, also one without halo rows of its own (its
            # rows may still be in other ranks' halos)
            if multi and shard.halo is not None:
                hl = shard.halo
                back, back_w = env.all_to_all_async(d_xext[n_own:].contiguous(), hl.recv_splits,
                                                    hl.send_splits)
        # the previous layer's post-table gradient is complete: its reduce-scatter starts now
        if prev_pm:
            if R_split is not None:
                R = R_split
            else:
                g = G_prev if G_prev is not None else hpo.new_zeros(shard.n_posts_pad,
                                                                     hpo.shape[1])
                R = env.reduce_scatter_async(g) if multi else (g, _Done())
            if jp is not None:
                R_proj = (proj[li][0], col_pre, pending_w)
        # B5 user rows' share of the post partial sums, then the halo rows' gradients
        for et, parts in gath.items():
            r = shard.rels[et]
            for hf, (full, w) in parts:       # the first range's K2 while the next one lands
                w.wait()
                if hf is None:
                    impl.weighted_scatter_bwd_raw(full, r.csr, r.w_bwd, out=d_hu)
                else:
                    impl.weighted_scatter_bwd_raw(full, hf.csr, hf.w_bwd, out=d_hu)
        if back is not None:
            back_w.wait()
            impl.scatter_mean_bwd_raw(back, shard.halo.rel_send, out=d_hu)
        G_u, G_full, G_own = d_hu, G_prev, d_hpo
    return loss


def sync_grads(model: torch.nn.Module, env: DistEnv, force: bool = False) -> None:
    """Sum parameter gradients over ranks with one flat all-reduce.  Every rank contributes every
    trainable parameter (zeros where its backward produced no gradient — a rank whose shard holds
    no edge of some relation), so the flat buffers line up across ranks.  One concatenation in,
    one multi-tensor copy out (not a copy kernel per parameter).  No host sync: the whole
    function can be recorded in a HIP graph over RCCL (``minibatch.CapturedStep``).  ``force``:
    issue the all-reduce at world size 1 too (rehearsal of the captured collective on one GPU)."""
    if env.world == 1 and not force:
        return
    params = [p for p in model.parameters() if p.requires_grad]
    flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                      for p in params])
    if env.world > 1:
        env.all_reduce_(flat)
    elif force:
        dist.all_reduce(flat, group=env.group)
    views = [v.view_as(p) for v, p in zip(torch.split(flat, [p.numel() for p in params]), params)]
    have = [i for i, p in enumerate(params) if p.grad is not None]
    if have:
        torch._foreach_copy_([params[i].grad for i in have], [views[i] for i in have])
    for i, p in enumerate(params):
        if p.grad is None:
            p.grad = views[i].clone()
