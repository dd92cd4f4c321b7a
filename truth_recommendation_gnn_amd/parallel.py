"""Multi-GPU hetero-SAGE: users sharded across ranks, posts replicated, RCCL all-reduce.

One process per GPU (``torch.distributed``, backend ``nccl`` = RCCL over xGMI).  The user <-> post
graph is partitioned by USER (contiguous id ranges, the 10x larger node type), and the post
TABLE by row slices:

* rank r owns users [lo_r, hi_r) and every engages edge whose user it owns, so
  - the user-destination aggregation (``rev_engages``: post -> user, mean over the user's
    in-edges) is complete on the owner — no exchange (it reads the all-gathered post table);
  - the post-destination aggregation (``engages``: user -> post) is a per-rank PARTIAL sum over
    the rank's edges, each edge pre-scaled by 1/deg_global(post) (K1 with per-edge weights);
* rank r also owns a slice of post rows: one reduce-scatter gives it the exact mean for its
  slice, the post projection (K3) runs on that slice only, and one all-gather rebuilds the full
  post table for the next layer's user side and for the loss.  A reduce-scatter + all-gather
  moves what one all-reduce does, and the post-side compute is divided by the world size instead
  of replicated;
* backward: the all-gather's adjoint is a reduce-scatter of the post-table gradient (the loss's
  dP and the user side's K2 output, both partial), the reduce-scatter's adjoint an all-gather of
  the slice gradients, which K2 (weights transposed) sends to the owned users; parameter gradients
  are summed over ranks with one flat all-reduce.
* the link loss is sharded the same way: rank r scores the positive edges of its users against
  the gathered post table; normalised by the GLOBAL edge count and mean(pos_weights), the
  per-rank losses add up to the reference loss (``train_gnn.py:259-281``).

Per step: reduce-scatter + all-gather per layer forward, reduce-scatter + all-gather for the
layer-2 post gradients and one reduce-scatter for the layer-1 post input gradient, plus the weight
gradients.  All are asynchronous: the forward ones overlap the user side of the same (or next)
layer; the gradient all-gather is handed on unfinished to its only consumer (K2's backward) so the
user-side backward autograd runs before it overlaps it.  The compute ops are injected
(``HipImpl`` here; the CPU gloo tests inject plain-torch ops to check the partitioning logic).
"""
from __future__ import annotations

import dataclasses
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from . import ops
from .graph import RelationCSR, relation_csr
from .nn import HeteroSAGE, _fused_weights
from .synth import ENGAGES, REV_ENGAGES

RELATIONS = [(REV_ENGAGES, 1.0), (ENGAGES, 1.0)]


@dataclasses.dataclass
class DistEnv:
    world: int = 1
    rank: int = 0
    group: Optional[object] = None

    @classmethod
    def from_torch(cls) -> "DistEnv":
        if dist.is_available() and dist.is_initialized():
            return cls(dist.get_world_size(), dist.get_rank())
        return cls()

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            dist.all_reduce(t, group=self.group)
        return t

    def post_slice(self, n: int) -> Tuple[int, int, int]:
        """(slice rows, lo, hi): rank r owns rows [r*S, r*S+S) of the table padded to world*S."""
        S = -(-n // self.world) if n else 0
        return S, self.rank * S, self.rank * S + S

    def _direct(self, t: torch.Tensor) -> bool:
        """RCCL, or gloo on host tensors (the CPU tests), run the tensor collectives as is; gloo
        on device tensors (a one-GPU rehearsal) goes through all-reduce / all_gather lists."""
        return dist.get_backend(self.group) == "nccl" or not t.is_cuda

    def reduce_scatter_async(self, full: torch.Tensor):
        """Sum over ranks of ``full`` [world*S, ...]; returns (this rank's slice [S, ...], work)."""
        S = full.shape[0] // self.world
        if self._direct(full):
            out = torch.empty((S,) + tuple(full.shape[1:]), dtype=full.dtype, device=full.device)
            work = dist.reduce_scatter_tensor(out, full, group=self.group, async_op=True)
            return out, _Held(work, full, out)
        t = full.clone()
        dist.all_reduce(t, group=self.group)
        return t[self.rank * S:(self.rank + 1) * S].clone(), _Done()

    def all_gather_async(self, own: torch.Tensor):
        """Concatenation over ranks of ``own`` [S, ...]; returns (full [world*S, ...], work)."""
        full = torch.empty((own.shape[0] * self.world,) + tuple(own.shape[1:]), dtype=own.dtype,
                           device=own.device)
        if self._direct(own):
            work = dist.all_gather_into_tensor(full, own, group=self.group, async_op=True)
            return full, _Held(work, own, full)
        dist.all_gather(list(full.chunk(self.world)), own, group=self.group)
        return full, _Done()

    def all_reduce_async(self, t: torch.Tensor):
        """Start an in-place all-reduce; ``.wait()`` on the result before reading ``t`` (with
        NCCL/RCCL that is a stream wait, so kernels enqueued in between overlap the collective)."""
        if self.world > 1:
            return _Held(dist.all_reduce(t, group=self.group, async_op=True), t)
        return _Done()


class _Done:
    def wait(self):
        return True


class _Held:
    """An async collective's Work plus references to its buffers until ``wait()`` (gloo's async
    ops do not keep a temporary input alive on their own)."""

    def __init__(self, work, *refs):
        self.work, self.refs = work, refs

    def wait(self):
        # gloo finishes an async collective by copying into the output at wait(); outside no_grad
        # autograd would record that copy on an output it already tracks and cut its graph
        with torch.no_grad():
            self.work.wait()
        self.refs = None
        return True


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


class _AllGather(torch.autograd.Function):
    """Concatenation of every rank's slice; adjoint: reduce-scatter of the gradient (waited at
    once: autograd may add it to the slice's other gradients)."""

    @staticmethod
    def forward(ctx, own, env: DistEnv, handle: "Pending"):
        ctx.env = env
        full, handle.work = env.all_gather_async(own.contiguous())
        return full

    @staticmethod
    def backward(ctx, g):
        out, work = ctx.env.reduce_scatter_async(g.contiguous())
        work.wait()
        return out, None, None


def user_range(n_users: int, world: int, rank: int) -> Tuple[int, int]:
    m = -(-n_users // world)
    lo = min(n_users, rank * m)
    return lo, min(n_users, lo + m)


class HipImpl:
    """The MI355X kernels behind the partitioned step."""

    # weighted_gather's backward awaits a gradient whose all-reduce is still in flight
    defer_grad = True

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
    def edge_bce_loss(U, P, pos, neg, n_total, cscale, neg_order="edge"):
        return ops.edge_bce_loss(U, P, pos, neg, None, neg_order=neg_order, check=False,
                                 n_edges_total=n_total, cscale=cscale)


class UserShard:
    """Static per-rank structures for the engages relation (and its reverse)."""

    def __init__(self, engage_edges: torch.Tensor, n_users: int, n_posts: int, env: DistEnv,
                 impl=None, pos_weights: Optional[torch.Tensor] = None):
        impl = impl or HipImpl()
        self.env, self.impl = env, impl
        self.n_users, self.n_posts = n_users, n_posts
        self.lo, self.hi = user_range(n_users, env.world, env.rank)
        u, p = engage_edges[0], engage_edges[1]
        self.mask = (u >= self.lo) & (u < self.hi)
        self.pos_local = torch.stack([u[self.mask] - self.lo, p[self.mask]]).contiguous()
        self.rev_local = self.pos_local.flip(0).contiguous()
        self.n_own = self.hi - self.lo
        self.num_edges_global = int(engage_edges.shape[1])
        # post table padded to world * S rows; rank r owns rows [r*S, r*S+S)
        self.post_rows, self.p_lo, self.p_hi = env.post_slice(n_posts)
        self.n_posts_pad = self.post_rows * env.world
        deg = torch.bincount(self.pos_local[1], minlength=self.n_posts_pad).to(torch.float32)
        env.all_reduce_(deg)
        self.inv_deg_post = torch.where(deg > 0, 1.0 / deg.clamp(min=1.0), torch.zeros_like(deg))
        self.rel_eng = impl.relation(self.pos_local, self.n_own, self.n_posts_pad)
        self.rel_rev = impl.relation(self.rev_local, self.n_posts_pad, self.n_own)
        self.w_eng_fwd = impl.edge_weights_fwd(self.rel_eng, self.inv_deg_post)
        self.w_eng_bwd = impl.edge_weights_bwd(self.rel_eng, self.inv_deg_post)
        self.cscale = None
        if pos_weights is not None:   # global mean of the interaction weights (static)
            s = torch.stack([pos_weights[self.mask].to(torch.float64).sum(),
                             torch.tensor(float(self.mask.sum()), dtype=torch.float64,
                                          device=pos_weights.device)])
            env.all_reduce_(s)
            self.cscale = (s[0] / s[1]).to(torch.float32)

    def local_edges_of(self, per_edge: torch.Tensor) -> torch.Tensor:
        """Slice a per-global-edge tensor (e.g. injected negatives) to this rank's edges."""
        return per_edge[self.mask]

    def forward(self, model: HeteroSAGE, x_user_own: torch.Tensor, x_post: torch.Tensor):
        """Partitioned forward of ``model``; returns (owned user embeddings, post embeddings of
        the whole padded table — rows >= n_posts are padding)."""
        impl, env = self.impl, self.env
        if x_post.shape[0] != self.n_posts_pad:
            x_post = torch.nn.functional.pad(x_post, (0, 0, 0, self.n_posts_pad - x_post.shape[0]))
        h_u, h_p = x_user_own, x_post
        h_p_own = x_post[self.p_lo:self.p_hi]
        gathered = None                       # in-flight all-gather of h_p
        defer = getattr(impl, "defer_grad", False)
        nu = "__".join(REV_ENGAGES)
        np_ = "__".join(ENGAGES)
        wts = dict(model.relations)
        for convs in model.layers:
            shapes = {"user": h_u, "post": h_p}
            Wu, bu = _fused_weights(convs, [(nu, REV_ENGAGES, wts[REV_ENGAGES])], shapes)
            Wp, bp = _fused_weights(convs, [(np_, ENGAGES, wts[ENGAGES])], shapes)
            # post partial sums first; their reduce-scatter is in flight during the user side
            s_post = impl.weighted_gather(h_u, self.rel_eng, self.w_eng_fwd, self.w_eng_bwd)
            if env.world == 1:
                a_post, pend = s_post, Pending()
            else:
                pend = Pending()
                a_post = _ReduceScatter.apply(s_post, env, pend, defer)
            if gathered is not None:          # the previous layer's all-gather of h_p
                gathered.wait()
                gathered = None
            a_user = impl.mean_gather(h_p, self.rel_rev)
            h_u_next = impl.fused_linear([a_user, h_u], Wu, bu, True)
            pend.wait()
            # the post projection runs on this rank's slice only
            h_p_own = impl.fused_linear([a_post, h_p_own], Wp, bp, True)
            if env.world == 1:
                h_p = h_p_own
            else:
                gathered = Pending()
                h_p = _AllGather.apply(h_p_own, env, gathered)
            h_u = h_u_next
        if gathered is not None:
            gathered.wait()
        return h_u, h_p

    def loss(self, h_u_own, h_p, neg_local, neg_order="edge"):
        """This rank's additive share of the reference loss."""
        if self.cscale is None:
            raise ValueError("UserShard built without pos_weights")
        return self.impl.edge_bce_loss(h_u_own, h_p, self.pos_local, neg_local,
                                       self.num_edges_global, self.cscale, neg_order=neg_order)


def sync_grads(model: torch.nn.Module, env: DistEnv) -> None:
    """Sum parameter gradients over ranks with one flat all-reduce."""
    if env.world == 1:
        return
    params = [p for p in model.parameters() if p.grad is not None]
    flat = torch.cat([p.grad.reshape(-1) for p in params])
    env.all_reduce_(flat)
    o = 0
    for p in params:
        n = p.numel()
        p.grad.copy_(flat[o:o + n].view_as(p))
        o += n
