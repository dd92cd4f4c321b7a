"""Autograd operators over the HIP kernels.

``hetero_layer`` is one full SAGE layer over every destination node type at once — the fused
form of ``WeightedRGCN.forward`` (``train_gnn.py:166-200``):

    y_dst = act( sum_r w_r * (mean_{src->dst} x_src @ W_l,r^T + b_r + x_dst @ W_r,r^T) )

computed as: K1 ``gather_mean`` per relation, then ONE K3 multi-segment MFMA linear per
destination over ``[aggr_1 .. aggr_R, x_dst]`` with the K-concatenated, relation-weighted
weights (built by torch ops on the parameters, so autograd routes the gradients back to the
reference's own per-conv parameters).  Backward: K3 dgrad/wgrad (ReLU mask fused), then K2
``scatter_mean_bwd`` accumulating straight into the source-feature gradients, so the per-type
gradient sums the reference's autograd would do with separate add kernels happen in-kernel.
"""
from __future__ import annotations

import contextlib
import dataclasses
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _native as N
from .graph import RelationCSR


def _check_f32(t: torch.Tensor, what: str) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"{what}: hgnn computes in fp32 (the reference dtype); got {t.dtype}")
    return t.contiguous()


# ----------------------------------------------------------------------------- kernel timing
class KernelTimer:
    """Records HIP events around every kernel call this module makes (on the current stream,
    the one the kernels are launched on), with each launch's algorithmic HBM bytes.  Used by
    bench.py inside its timed region; ``None`` when off (zero overhead)."""

    def __init__(self):
        # (name, algorithmic bytes, start event, end event, compulsory bytes, flops)
        self.records = []

    def summary(self):
        torch.cuda.synchronize()
        agg = {}
        for name, nbytes, s, e, cbytes, flops in self.records:
            ms = s.elapsed_time(e)
            a = agg.setdefault(name, {"launches": 0, "ms": 0.0, "bytes": 0, "cbytes": 0,
                                      "flops": 0})
            a["launches"] += 1
            a["ms"] += ms
            a["bytes"] += nbytes
            a["cbytes"] += cbytes
            a["flops"] += flops
        return agg


_timer: Optional[KernelTimer] = None


def set_timer(t: Optional[KernelTimer]) -> None:
    global _timer
    _timer = t


class _timed:
    """``cbytes``: compulsory bytes (every table row counted once), when it differs from the
    algorithmic figure — the honest number for a gather whose source table is cache-resident.
    ``flops``: algorithmic flops of an MFMA kernel (K3), 0 elsewhere."""

    def __init__(self, name, nbytes, cbytes=None, flops=0):
        self.name, self.nbytes, self.flops = name, nbytes, flops
        self.cbytes = nbytes if cbytes is None else cbytes

    def __enter__(self):
        if _timer is not None:
            self.s = torch.cuda.Event(enable_timing=True)
            self.s.record()
        return self

    def __exit__(self, *exc):
        if _timer is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            _timer.records.append((self.name, int(self.nbytes), self.s, e, int(self.cbytes),
                                   int(self.flops)))


def gather_bytes(n_edges: int, n_rows: int, d: int, weighted: bool) -> int:
    """Algorithmic HBM bytes of one K1/K2 launch: per edge a 4-B index and one
    4*d-B source row (+4 B weight for K2), rowptr, and the output rows."""
    return 4 * n_edges * (1 + d + (1 if weighted else 0)) + 4 * (n_rows + 1) + 4 * n_rows * d


def gather_compulsory_bytes(n_edges: int, n_rows: int, n_src: int, d: int, weighted: bool) -> int:
    """As gather_bytes with each source row read once: min(E, N_src) rows instead of E."""
    return (4 * n_edges * (1 + (1 if weighted else 0)) + 4 * min(n_edges, n_src) * d
            + 4 * (n_rows + 1) + 4 * n_rows * d)


# ----------------------------------------------------------------------------- raw kernel calls
# Source-blocked gathers.  Random rows from a table of several GB come back at ~6.3 TB/s; the
# same rows from a ~600 MB slice of it at ~7.2 TB/s (cfg4 K1 post<-user, scripts/ic_block_bench.py:
# 16.96 ms in one pass, 15.36 ms in 8 passes over 575-MB user blocks, each pass adding its block's
# sum into the output).  The passes re-read and re-write the output (B-1 extra round trips of
# N_dst x 4d bytes), which the gain pays for only while the blocks stay large: 8 passes is the
# best measured split of a 4.6 GB table, 16 is already even.  So a gather whose source table is
# at least GATHER_BLOCK_BYTES is split into ceil(table / GATHER_BLOCK_SLICE) passes.
GATHER_BLOCK_BYTES = int(float(os.environ.get("HGNN_GATHER_BLOCK_GB", "2")) * 2**30)
GATHER_BLOCK_SLICE = int(float(os.environ.get("HGNN_GATHER_BLOCK_MB", "600")) * 2**20)


def gather_blocks(x: torch.Tensor, n_edges: Optional[int] = None) -> int:
    """Number of source-block passes for a gather reading table ``x`` (1: one plain pass).  A
    gather of fewer edges than the table has rows (a sampled block reading the global tables)
    reads a thin random subset at latency-bound rates, where the passes' locality buys nothing
    and their (block, row) CSR would cost a sort per block: one pass."""
    nbytes = x.numel() * x.element_size()
    if GATHER_BLOCK_BYTES <= 0 or nbytes < GATHER_BLOCK_BYTES:
        return 1
    if n_edges is not None and n_edges < x.shape[0]:
        return 1
    return int(-(-nbytes // GATHER_BLOCK_SLICE))


def _gather_blocked(x, passes, row_w, edge_w, out, accumulate, name, nbytes, cbytes):
    """All passes of a source-blocked gather, timed as one gather (its algorithmic bytes are the
    unblocked gather's)."""
    dev = out.device
    d = int(out.shape[1])
    lib, s = N.lib(), N.stream_ptr(dev)
    with _timed(name, nbytes, cbytes):
        for b, g in enumerate(passes):
            p = g.plan
            slab = (torch.empty(p.n_chunks * d, dtype=torch.float32, device=dev)
                    if p.n_heavy else None)
            flags = N.HGNN_ACCUMULATE if (accumulate or b > 0) else 0
            N.check(lib.hgnn_gather_reduce_scaled(
                N.ptr(x), x.shape[0], d, N.ptr(g.rowptr), N.ptr(g.col), g.n_rows, N.ptr(edge_w),
                None, N.ptr(row_w), flags, N.ptr(p.heavy_rows), N.ptr(p.heavy_first), p.n_heavy,
                p.n_chunks, p.chunk, N.ptr(slab), N.ptr(out), s), "hgnn_gather_reduce_scaled")


def gather_mean(x_src: torch.Tensor, csr: RelationCSR,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K1: ``aggr[i] = mean_{(j->i)} x_src[j]`` (0 for an empty row); added into ``out`` when
    given."""
    x_src = _check_f32(x_src, "gather_mean")
    dev = N.require_device(x_src, csr.fwd.rowptr)
    if x_src.shape[0] != csr.n_src:
        raise ValueError(f"x_src has {x_src.shape[0]} rows, relation expects {csr.n_src}")
    d = int(x_src.shape[1])
    acc = out is not None
    if out is None:
        out = torch.empty(csr.n_dst, d, dtype=torch.float32, device=dev)
    B = gather_blocks(x_src, csr.num_edges) if csr.num_edges else 1
    if B > 1:
        passes, _ = csr.blocks("fwd", B)
        E = csr.num_edges
        _gather_blocked(x_src, passes, csr.inv_deg, None, out, acc,
                        f"gather_fwd[{csr.n_dst}<-{csr.n_src}]x{d}",
                        gather_bytes(E, csr.n_dst, d, False),
                        gather_compulsory_bytes(E, csr.n_dst, csr.n_src, d, False))
        return out
    _gather(x_src, csr.fwd, None, csr_mean=True, out=out, accumulate=acc)
    return out


def _multi_ok(jobs) -> bool:
    """Whether gathers (x, grouped, out) can share one ``hgnn_gather_reduce_multi`` launch:
    2..8 of them, no heavy-row plan, one fp32 row width (a multiple of 4, <= 512), distinct
    outputs, and no per-kernel timer running (its events time each relation's launch)."""
    if _timer is not None or not 2 <= len(jobs) <= 8:
        return False
    d = int(jobs[0][2].shape[1])
    outs = {o.data_ptr() for _, _, o in jobs}
    return (len(outs) == len(jobs) and d % 4 == 0 and d <= 512 and
            all(g.plan.n_heavy == 0 and int(o.shape[1]) == d and x.dtype == torch.float32
                for x, g, o in jobs))


def _gather_multi(jobs, mean: bool, accumulate: bool, edge_ws=None, acc_limit=None) -> None:
    """``_gather`` of every (x, grouped, out) job in one launch (see ``_multi_ok``);
    ``acc_limit[j]`` > 0: job j accumulates only into its rows below it."""
    dev = jobs[0][2].device
    flags = (N.HGNN_MEAN if mean else 0) | (N.HGNN_ACCUMULATE if accumulate else 0)
    N.check(N.lib().hgnn_gather_reduce_multi(
        len(jobs), N.ptr_array([x for x, _, _ in jobs]),
        N.i64_array([int(x.shape[0]) for x, _, _ in jobs]), int(jobs[0][2].shape[1]),
        N.ptr_array([g.rowptr for _, g, _ in jobs]), N.ptr_array([g.col for _, g, _ in jobs]),
        N.i64_array([g.n_rows for _, g, _ in jobs]),
        N.ptr_array(edge_ws) if edge_ws is not None else None, flags,
        N.i64_array(acc_limit) if acc_limit is not None else None,
        N.ptr_array([o for _, _, o in jobs]), N.stream_ptr(dev)), "hgnn_gather_reduce_multi")


def gather_mean_many(pairs: Sequence[Tuple[torch.Tensor, RelationCSR]]) -> List[torch.Tensor]:
    """``gather_mean(x, csr)`` of every pair — one launch for all of them when they qualify
    (sampled blocks: short rows, one pass each; ``_multi_ok``), else one call each."""
    jobs = []
    for x, csr in pairs:
        x = _check_f32(x, "gather_mean")
        if x.shape[0] != csr.n_src:
            raise ValueError(f"x_src has {x.shape[0]} rows, relation expects {csr.n_src}")
        if csr.num_edges and gather_blocks(x, csr.num_edges) > 1:
            return [gather_mean(x, c) for x, c in pairs]
        jobs.append((x, csr.fwd, torch.empty(csr.n_dst, int(x.shape[1]), dtype=torch.float32,
                                             device=x.device)))
    if not _multi_ok(jobs):
        return [gather_mean(x, c) for x, c in pairs]
    _gather_multi(jobs, mean=True, accumulate=False)
    return [o for _, _, o in jobs]


def _gather(x, grouped, col_w, csr_mean, out, accumulate, edge_w=None, kind=None):
    p = grouped.plan
    dev = out.device
    slab = None
    if p.n_heavy:
        slab = torch.empty(p.n_chunks * out.shape[1], dtype=torch.float32, device=dev)
    flags = (N.HGNN_MEAN if csr_mean else 0) | (N.HGNN_ACCUMULATE if accumulate else 0)
    d = int(out.shape[1])
    weighted = edge_w is not None or col_w is not None
    kind = kind or ("fwd" if csr_mean else "bwd")   # "wfwd": weighted forward (parallel.py)
    name = f"gather_{kind}[{grouped.n_rows}<-{x.shape[0]}]x{d}"   # [dst rows <- src rows] x d
    E = int(grouped.col.numel())
    with _timed(name, gather_bytes(E, grouped.n_rows, d, weighted),
                gather_compulsory_bytes(E, grouped.n_rows, int(x.shape[0]), d, weighted)):
        N.check(N.lib().hgnn_gather_reduce(
            N.ptr(x), x.shape[0], d, N.ptr(grouped.rowptr), N.ptr(grouped.col),
            grouped.n_rows, N.ptr(edge_w), N.ptr(col_w), flags, N.ptr(p.heavy_rows),
            N.ptr(p.heavy_first), p.n_heavy, p.n_chunks, p.chunk, N.ptr(slab), N.ptr(out),
            N.stream_ptr(dev)), "hgnn_gather_reduce")


def _score_gather(U, P, grouped, mode, cscale, inv_e, out, accumulate, tag):
    """dP rows from the loss: each edge's weight recomputed from <U[u], P[row]> (mode 1 positive,
    2 negative) inside the gather — see hgnn_score_gather."""
    p = grouped.plan
    dev = out.device
    d = int(out.shape[1])
    slab = None
    if p.n_heavy:
        slab = torch.empty(p.n_chunks * d, dtype=torch.float32, device=dev)
    E = int(grouped.col.numel())
    nb = gather_bytes(E, grouped.n_rows, d, False) + 4 * grouped.n_rows * d
    cb = (gather_compulsory_bytes(E, grouped.n_rows, int(U.shape[0]), d, False)
          + 4 * grouped.n_rows * d)
    with _timed(f"score_gather_{tag}[{grouped.n_rows}<-{U.shape[0]}]x{d}", nb, cb):
        N.check(N.lib().hgnn_score_gather(
            N.ptr(U), U.shape[0], N.ptr(P), d, N.ptr(grouped.rowptr), N.ptr(grouped.col),
            grouped.n_rows, mode, N.ptr(cscale), inv_e, N.ptr(p.heavy_rows), N.ptr(p.heavy_first),
            p.n_heavy, p.n_chunks, p.chunk, N.ptr(slab), N.ptr(out), 1 if accumulate else 0,
            N.stream_ptr(dev)), "hgnn_score_gather")


def _score_gather2(U, P, pos, negs, cscale, inv_e, out):
    """Both dP gathers in one pass (hgnn_score_gather2): row r sums its positive edges (mode 1,
    heavy-row plan) and its negatives (mode 2) into one accumulator and writes dP[r] once."""
    p = pos.plan
    dev = out.device
    d = int(out.shape[1])
    n = pos.n_rows
    slab = None
    if p.n_heavy:
        slab = torch.empty(p.n_chunks * d, dtype=torch.float32, device=dev)
    E = int(pos.col.numel()) + int(negs.col.numel())
    nb = gather_bytes(E, n, d, False) + 4 * (n + 1) + 4 * n * d
    cb = gather_compulsory_bytes(E, n, int(U.shape[0]), d, False) + 4 * (n + 1) + 4 * n * d
    with _timed(f"score_gather[{n}<-{U.shape[0]}]x{d}", nb, cb):
        N.check(N.lib().hgnn_score_gather2(
            N.ptr(U), U.shape[0], N.ptr(P), d, N.ptr(pos.rowptr), N.ptr(pos.col),
            N.ptr(negs.rowptr), N.ptr(negs.col), n, N.ptr(cscale), inv_e, N.ptr(p.heavy_rows),
            N.ptr(p.heavy_first), p.n_heavy, p.n_chunks, p.chunk, N.ptr(slab), N.ptr(out),
            N.stream_ptr(dev)), "hgnn_score_gather2")


def scatter_mean_bwd(grad_aggr: torch.Tensor, csr: RelationCSR,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K2: ``grad_x_src[j] (+)= sum_{(j->i)} grad_aggr[i] / deg_i`` over the CSC."""
    grad_aggr = _check_f32(grad_aggr, "scatter_mean_bwd")
    dev = grad_aggr.device
    d = int(grad_aggr.shape[1])
    acc = out is not None
    if out is None:
        out = torch.empty(csr.n_src, d, dtype=torch.float32, device=dev)
    B = gather_blocks(grad_aggr, csr.num_edges) if csr.num_edges else 1
    if B > 1:
        passes, w = csr.blocks("bwd", B)
        E = csr.num_edges
        _gather_blocked(grad_aggr, passes, None, w, out, acc,
                        f"gather_bwd[{csr.n_src}<-{csr.n_dst}]x{d}",
                        gather_bytes(E, csr.n_src, d, True),
                        gather_compulsory_bytes(E, csr.n_src, csr.n_dst, d, True))
        return out
    _gather(grad_aggr, csr.bwd, None, csr_mean=False, out=out, accumulate=acc,
            edge_w=csr.bwd_weights)
    return out


def relu_mask_for(n: int, h: int, relu: bool, dev, k: Optional[int] = None
                  ) -> Optional[torch.Tensor]:
    """The bit form of a K3 output's ReLU mask (``hgnn_linear_fwd_mask``: 16 B per row, the
    backward reads it instead of the 4h-byte output), or None where the kernels have no bit form
    (no ReLU, h not a multiple of 16 or above 128, or ``HGNN_RELU_BITS=0``) or where no kernel
    would read it: an input width ``k`` outside the persistent kernels' {64, 128, 256} (the
    general kernels read the output, and the bits would cost a separate launch)."""
    if not (RELU_BITS and relu and h % 16 == 0 and h <= 128):
        return None
    if k is not None and k not in (64, 128, 256):
        return None
    return torch.empty((n, 4), dtype=torch.int32, device=dev)


RELU_BITS = os.environ.get("HGNN_RELU_BITS", "1") == "1"


def _check_rows(segs, n, what):
    """Every segment of a K3 call has the same n rows (the kernels read each without bounds)."""
    for i, s_ in enumerate(segs):
        if s_.dim() != 2 or int(s_.shape[0]) != n:
            raise ValueError(f"{what}: segment {i} is {tuple(s_.shape)}, expected {n} rows")


def linear_fwd(segs: Sequence[torch.Tensor], w: torch.Tensor, b: Optional[torch.Tensor],
               relu: bool, add: Optional[torch.Tensor] = None,
               mask_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K3/K4: ``act(sum_s segs[s] @ w[:, seg s]^T + b (+ add))``; ``mask_out`` (from
    :func:`relu_mask_for`) also receives the ReLU mask as bits."""
    n = int(segs[0].shape[0])
    h = int(w.shape[0])
    ks = [int(s.shape[1]) for s in segs]
    if w.shape[1] != sum(ks):
        raise ValueError(f"weight has {w.shape[1]} input columns, segments sum to {sum(ks)}")
    _check_rows(segs, n, "linear_fwd")
    if add is not None and tuple(add.shape) != (n, h):
        raise ValueError(f"linear_fwd: add is {tuple(add.shape)}, expected {(n, h)}")
    if b is not None and b.numel() != h:
        raise ValueError(f"linear_fwd: bias has {b.numel()} entries, expected {h}")
    dev = w.device
    out = torch.empty(n, h, dtype=torch.float32, device=dev)
    k = sum(ks)
    nb = 4 * n * (k + h + (h if add is not None else 0)) + (16 * n if mask_out is not None else 0)
    with _timed(f"linear_fwd[{n}x{k}->{h}]", nb, flops=2 * n * k * h):
        N.check(N.lib().hgnn_linear_fwd_mask(len(segs), N.ptr_array(segs), N.int_array(ks), n,
                                             N.ptr(w), h, N.ptr(b), N.ptr(add),
                                             1 if relu else 0, N.ptr(out), N.ptr(mask_out),
                                             N.stream_ptr(dev)), "hgnn_linear_fwd_mask")
    return out


def linear_bwd(segs, w, dout, out_act, dxs: Sequence[Optional[torch.Tensor]], need_w: bool,
               need_b: bool, dz_out: Optional[torch.Tensor] = None,
               mask: Optional[torch.Tensor] = None, dx_add: Sequence[bool] = ()):
    """K3 backward; ``dz_out`` (optional [n, h]) receives the masked dz as well; ``mask``: the
    forward's ReLU bits (read instead of ``out_act`` by the persistent kernels); ``dx_add[s]``:
    segment s's input gradient is added into what ``dxs[s]`` holds (``hgnn_linear_bwd_ex``)."""
    n = int(segs[0].shape[0])
    h = int(w.shape[0])
    ks = [int(s.shape[1]) for s in segs]
    if w.shape[1] != sum(ks):
        raise ValueError(f"weight has {w.shape[1]} input columns, segments sum to {sum(ks)}")
    _check_rows(segs, n, "linear_bwd")
    for what, t in (("dout", dout), ("out_act", out_act), ("dz_out", dz_out)):
        if t is not None and tuple(t.shape) != (n, h):
            raise ValueError(f"linear_bwd: {what} is {tuple(t.shape)}, expected {(n, h)}")
    if len(dxs) != len(segs):
        raise ValueError(f"linear_bwd: {len(dxs)} dx buffers for {len(segs)} segments")
    for s_, dx in zip(segs, dxs):
        if dx is not None and tuple(dx.shape) != tuple(s_.shape):
            raise ValueError(f"linear_bwd: dx {tuple(dx.shape)} for a {tuple(s_.shape)} segment")
    if mask is not None and tuple(mask.shape) != (n, 4):
        raise ValueError(f"linear_bwd: ReLU bits are {tuple(mask.shape)}, expected {(n, 4)}")
    dev = w.device
    dw = torch.empty_like(w) if need_w else None
    db = torch.empty(h, dtype=torch.float32, device=dev) if need_b else None
    ws = None
    if need_w or need_b:
        ws = N.workspace(N.lib().hgnn_linear_bwd_ws_bytes(n, sum(ks), h), dev)
    k_dx = sum(k for k, dx in zip(ks, dxs) if dx is not None)
    bits = mask is not None and out_act is not None
    nb = 4 * n * (h + (h if out_act is not None and not bits else 0) + sum(ks) + k_dx) + \
        (16 * n if bits else 0) + (4 * n * h if dz_out is not None else 0)
    fl = 2 * n * h * k_dx + (2 * n * sum(ks) * h if need_w else 0)   # dgrad + wgrad
    acc = 0
    for i, on in enumerate(dx_add):
        if on and dxs[i] is not None:
            acc |= 1 << i
            nb += 4 * n * ks[i]          # the gradient already there is read back
    with _timed(f"linear_bwd[{n}x{sum(ks)}->{h}]", nb, flops=fl):
        N.check(N.lib().hgnn_linear_bwd_ex(
            len(segs), N.ptr_array(segs), N.int_array(ks), n, N.ptr(w), h, N.ptr(dout),
            N.ptr(out_act), N.ptr(mask if out_act is not None else None), N.ptr_array(dxs),
            acc, N.ptr(dw), N.ptr(db), N.ptr(dz_out), N.ptr(ws), 0 if ws is None else ws.numel(),
            N.stream_ptr(dev)), "hgnn_linear_bwd_ex")
    return dw, db


def linear_fwd_many(jobs) -> List[torch.Tensor]:
    """:func:`linear_fwd` (no ``add``) of each ``(segs, w, b, relu, mask_out)`` job in one native
    call (``hgnn_linear_fwd_multi``): a sampled layer's two destination types on the K = 384 /
    512 split path share each column block's launch; anything else runs job by job there."""
    if len(jobs) == 1 or len({int(j[1].shape[0]) for j in jobs}) > 1:   # (one output width)
        return [linear_fwd(segs, w, b, relu, mask_out=mk) for segs, w, b, relu, mk in jobs]
    outs, n_seg, xs, ks, rows, ws_, bs, relus, mks = [], [], [], [], [], [], [], [], []
    nb = fl = 0
    for segs, w, b, relu, mk in jobs:
        n, h = int(segs[0].shape[0]), int(w.shape[0])
        k = [int(s_.shape[1]) for s_ in segs]
        if w.shape[1] != sum(k):
            raise ValueError(f"weight has {w.shape[1]} input columns, segments sum to {sum(k)}")
        _check_rows(segs, n, "linear_fwd_many")
        if b is not None and b.numel() != h:
            raise ValueError(f"linear_fwd_many: bias has {b.numel()} entries, expected {h}")
        out = torch.empty(n, h, dtype=torch.float32, device=w.device)
        outs.append(out)
        n_seg.append(len(segs)); xs.extend(segs); ks.extend(k); rows.append(n)
        ws_.append(w); bs.append(b); relus.append(1 if relu else 0); mks.append(mk)
        nb += 4 * n * (sum(k) + h) + (16 * n if mk is not None else 0)
        fl += 2 * n * sum(k) * h
    dev = jobs[0][1].device
    h = int(jobs[0][1].shape[0])
    with _timed(f"linear_fwd_multi[{'+'.join(str(r) for r in rows)}x{sum(ks) // len(jobs)}->{h}]",
                nb, flops=fl):
        N.check(N.lib().hgnn_linear_fwd_multi(
            len(jobs), N.int_array(n_seg), N.ptr_array(xs), N.int_array(ks), N.i64_array(rows),
            N.ptr_array(ws_), h, N.ptr_array(bs), N.int_array(relus), N.ptr_array(outs),
            N.ptr_array(mks), N.stream_ptr(dev)), "hgnn_linear_fwd_multi")
    return outs


def linear_bwd_many(jobs):
    """:func:`linear_bwd` (no ``dz_out``, no ``dx_add``) of each ``(segs, w, dout, out_act, dxs,
    need_w, need_b, mask)`` job in one native call (``hgnn_linear_bwd_multi``); returns the
    ``(dw, db)`` of each."""
    if len(jobs) == 1 or len({int(j[1].shape[0]) for j in jobs}) > 1:
        return [linear_bwd(segs, w, dout, out_act, dxs, need_w, need_b, mask=mk)
                for segs, w, dout, out_act, dxs, need_w, need_b, mk in jobs]
    n_seg, xs, ks, rows, kt, ws_, douts, outs, mks, dxs_all, dws, dbs = ([] for _ in range(12))
    nb = fl = 0
    h = int(jobs[0][1].shape[0])
    for segs, w, dout, out_act, dxs, need_w, need_b, mk in jobs:
        n = int(segs[0].shape[0])
        k = [int(s_.shape[1]) for s_ in segs]
        if w.shape[1] != sum(k):
            raise ValueError(f"weight has {w.shape[1]} input columns, segments sum to {sum(k)}")
        _check_rows(segs, n, "linear_bwd_many")
        for what, t in (("dout", dout), ("out_act", out_act)):
            if t is not None and tuple(t.shape) != (n, h):
                raise ValueError(f"linear_bwd_many: {what} is {tuple(t.shape)}, expected {(n, h)}")
        if len(dxs) != len(segs):
            raise ValueError(f"linear_bwd_many: {len(dxs)} dx buffers for {len(segs)} segments")
        for s_, dx in zip(segs, dxs):
            if dx is not None and tuple(dx.shape) != tuple(s_.shape):
                raise ValueError(f"linear_bwd_many: dx {tuple(dx.shape)} for a "
                                 f"{tuple(s_.shape)} segment")
        if mk is not None and tuple(mk.shape) != (n, 4):
            raise ValueError(f"linear_bwd_many: ReLU bits are {tuple(mk.shape)}, expected {(n, 4)}")
        n_seg.append(len(segs)); xs.extend(segs); ks.extend(k); rows.append(n); kt.append(sum(k))
        ws_.append(w); douts.append(dout); outs.append(out_act)
        mks.append(mk if out_act is not None else None); dxs_all.extend(dxs)
        dws.append(torch.empty_like(w) if need_w else None)
        dbs.append(torch.empty(h, dtype=torch.float32, device=w.device) if need_b else None)
        k_dx = sum(kk for kk, dx in zip(k, dxs) if dx is not None)
        bits = mk is not None and out_act is not None
        nb += 4 * n * (h + (h if out_act is not None and not bits else 0) + sum(k) + k_dx) + \
            (16 * n if bits else 0)
        fl += 2 * n * h * k_dx + (2 * n * sum(k) * h if need_w else 0)
    dev = jobs[0][1].device
    ws = None
    if any(d is not None for d in dws + dbs):
        ws = N.workspace(N.lib().hgnn_linear_bwd_multi_ws_bytes(
            len(jobs), N.i64_array(rows), N.int_array(kt), h), dev)
    with _timed(f"linear_bwd_multi[{'+'.join(str(r) for r in rows)}x{sum(kt) // len(jobs)}->{h}]",
                nb, flops=fl):
        N.check(N.lib().hgnn_linear_bwd_multi(
            len(jobs), N.int_array(n_seg), N.ptr_array(xs), N.int_array(ks), N.i64_array(rows),
            N.ptr_array(ws_), h, N.ptr_array(douts), N.ptr_array(outs), N.ptr_array(mks),
            N.ptr_array(dxs_all), None, N.ptr_array(dws), N.ptr_array(dbs), N.ptr(ws),
            0 if ws is None else ws.numel(), N.stream_ptr(dev)), "hgnn_linear_bwd_multi")
    return list(zip(dws, dbs))


# ----------------------------------------------------------------------------- fused weights
def split_weight_grads(dW: torch.Tensor, db: Optional[torch.Tensor], ks: Sequence[int],
                       k_root: int, scales: Sequence[float],
                       dwl: Sequence[Optional[torch.Tensor]], dwr: Sequence[Optional[torch.Tensor]],
                       dbl: Sequence[Optional[torch.Tensor]], plan=None) -> None:
    """Adjoint of :func:`fuse_weights` into the given gradient buffers (entries may be None):
    dwl[r] = s_r dW[:, block r], dwr[r] = s_r dW[:, root], dbl[r] = s_r db (one launch)."""
    dev = dW.device
    a_ks = plan.a_ks if plan is not None else N.int_array(ks)
    a_sc = plan.a_sc if plan is not None else N.float_array(scales)
    N.check(N.lib().hgnn_split_weight_grads(
        len(ks), N.ptr(dW.contiguous()), N.ptr(None if db is None else db.contiguous()),
        a_ks, int(k_root), a_sc, int(dW.shape[0]),
        N.ptr_array(dwl), N.ptr_array(dwr), N.ptr_array(dbl), N.stream_ptr(dev)),
        "hgnn_split_weight_grads")


class _FusePlan:
    """The host side of one fused-weight launch, built once per set of parameter buffers: the
    layout (meta) and the ctypes argument arrays.  Parameters keep their storage across
    optimizer steps, so a sampled mini-batch step (four of these per step at cfg5, where the
    host issue time is the step time) reuses them instead of rebuilding them per call."""
    __slots__ = ("meta", "a_wl", "a_wr", "a_bl", "a_ks", "a_sc")

    def __init__(self, meta, wl, wr, bl):
        ks, k_root, scales, _, _ = meta
        self.meta = meta
        self.a_wl, self.a_wr, self.a_bl = N.ptr_array(wl), N.ptr_array(wr), N.ptr_array(bl)
        self.a_ks, self.a_sc = N.int_array(ks), N.float_array(scales)


_FUSE_PLANS: "Dict[tuple, _FusePlan]" = {}


def _fuse_plan(meta, wl, wr, bl) -> _FusePlan:
    ts = [t for t in (*wl, *wr, *bl) if t is not None]
    if not all(t.is_contiguous() for t in ts):
        return _FusePlan(meta, [t.contiguous() for t in wl],
                         [None if t is None else t.contiguous() for t in wr],
                         [None if t is None else t.contiguous() for t in bl])
    key = (meta, tuple(0 if t is None else t.data_ptr() for t in (*wl, *wr, *bl)))
    plan = _FUSE_PLANS.get(key)
    if plan is None:
        if len(_FUSE_PLANS) >= 1024:
            _FUSE_PLANS.clear()
        plan = _FUSE_PLANS[key] = _FusePlan(meta, wl, wr, bl)
    return plan


class _FuseWeights(torch.autograd.Function):
    """``[s_1 Wl_1 | ... | s_R Wl_R | sum_r s_r Wr_r]`` and ``sum_r s_r bl_r`` in one launch
    (``hgnn_fuse_weights``); backward: every parameter's gradient in one launch."""

    @staticmethod
    def forward(ctx, meta, *ts):
        ks, k_root, scales, has_r, has_b = meta
        R = len(ks)
        wl, it = list(ts[:R]), iter(ts[R:])
        wr = [next(it) if hr else None for hr in has_r]
        bl = [next(it) if hb else None for hb in has_b]
        h, dev = int(wl[0].shape[0]), wl[0].device
        W = torch.empty(h, sum(ks) + k_root, dtype=torch.float32, device=dev)
        b = torch.empty(h, dtype=torch.float32, device=dev) if any(has_b) else None
        plan = _fuse_plan(meta, wl, wr, bl)
        N.check(N.lib().hgnn_fuse_weights(R, plan.a_wl, plan.a_ks, plan.a_wr, int(k_root),
                                          plan.a_bl, plan.a_sc, h, N.ptr(W), N.ptr(b),
                                          N.stream_ptr(dev)), "hgnn_fuse_weights")
        ctx.meta, ctx.h, ctx.dev, ctx.plan = meta, h, dev, plan
        return (W, b) if b is not None else W

    @staticmethod
    def backward(ctx, dW, db=None):
        ks, k_root, scales, has_r, has_b = ctx.meta
        R = len(ks)
        need = ctx.needs_input_grad[1:]
        new = lambda shape, i: (torch.empty(shape, dtype=torch.float32, device=ctx.dev)
                                if need[i] else None)
        dwl = [new((ctx.h, k), r) for r, k in enumerate(ks)]
        i = R
        dwr, dbl = [], []
        for hr in has_r:
            dwr.append(new((ctx.h, k_root), i) if hr else None)
            i += hr
        for hb in has_b:
            dbl.append(new((ctx.h,), i) if hb else None)
            i += hb
        if dW is None:
            dW = torch.zeros(ctx.h, sum(ks) + k_root, dtype=torch.float32, device=ctx.dev)
        split_weight_grads(dW, db if any(has_b) else None, ks, k_root, scales, dwl, dwr, dbl,
                           plan=ctx.plan)
        return (None, *dwl, *[t for t, hr in zip(dwr, has_r) if hr],
                *[t for t, hb in zip(dbl, has_b) if hb])


def fuse_weights(wl: Sequence[torch.Tensor], wr: Sequence[Optional[torch.Tensor]],
                 bl: Sequence[Optional[torch.Tensor]], scales: Sequence[float]
                 ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Differentiable fused weight of a destination update (see ``hgnn_fuse_weights``)."""
    ks = tuple(int(t.shape[1]) for t in wl)
    roots = [t for t in wr if t is not None]
    k_root = int(roots[0].shape[1]) if roots else 0
    meta = (ks, k_root, tuple(float(x) for x in scales), tuple(t is not None for t in wr),
            tuple(t is not None for t in bl))
    out = _FuseWeights.apply(meta, *wl, *roots, *[t for t in bl if t is not None])
    return out if isinstance(out, tuple) else (out, None)


class _FuseWeightsMulti(torch.autograd.Function):
    """``_FuseWeights`` for every destination update of a layer in one launch each way
    (``hgnn_fuse_weights_multi`` / ``hgnn_split_weight_grads_multi``): a layer's updates cost
    one fuse and one split launch instead of one each per update."""

    @staticmethod
    def forward(ctx, metas, *ts):
        h, dev = int(ts[0].shape[0]), ts[0].device
        outs, w_out, b_out, groups, i = [], [], [], [], 0
        for meta in metas:
            ks, k_root, scales, has_r, has_b = meta
            R = len(ks)
            n = R + sum(has_r) + sum(has_b)
            g = ts[i:i + n]
            i += n
            wl, it = list(g[:R]), iter(g[R:])
            wr = [next(it) if hr else None for hr in has_r]
            bl = [next(it) if hb else None for hb in has_b]
            groups.append((wl, wr, bl))
            W = torch.empty(h, sum(ks) + k_root, dtype=torch.float32, device=dev)
            b = torch.empty(h, dtype=torch.float32, device=dev) if any(has_b) else None
            w_out.append(W)
            b_out.append(b)
            outs.append(W)
            if b is not None:
                outs.append(b)
        plan = _fuse_multi_plan(metas, groups)
        N.check(N.lib().hgnn_fuse_weights_multi(
            len(metas), plan.a_nrel, plan.a_wl, plan.a_ks, plan.a_wr, plan.a_kroot, plan.a_bl,
            plan.a_sc, h, N.ptr_array(w_out), N.ptr_array(b_out), N.stream_ptr(dev)),
            "hgnn_fuse_weights_multi")
        ctx.metas, ctx.h, ctx.dev, ctx.plan = metas, h, dev, plan
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        need = ctx.needs_input_grad[1:]
        dws, dbs, dwl, dwr, dbl, ret = [], [], [], [], [], []
        gi = ni = 0
        for meta in ctx.metas:
            ks, k_root, scales, has_r, has_b = meta
            dW = grads[gi]
            gi += 1
            db = None
            if any(has_b):
                db = grads[gi]
                gi += 1
            if dW is None:
                dW = torch.zeros(ctx.h, sum(ks) + k_root, dtype=torch.float32, device=ctx.dev)
            if db is None and any(has_b):
                db = torch.zeros(ctx.h, dtype=torch.float32, device=ctx.dev)
            dws.append(dW.contiguous())
            dbs.append(None if db is None else db.contiguous())
            new = lambda shape, j: (torch.empty(shape, dtype=torch.float32, device=ctx.dev)
                                    if need[j] else None)
            gl = [new((ctx.h, k), ni + r) for r, k in enumerate(ks)]
            j = ni + len(ks)
            gr, gb = [], []
            for hr in has_r:
                gr.append(new((ctx.h, k_root), j) if hr else None)
                j += hr
            for hb in has_b:
                gb.append(new((ctx.h,), j) if hb else None)
                j += hb
            ni = j
            dwl += gl
            dwr += gr
            dbl += gb
            ret += gl + [t for t, hr in zip(gr, has_r) if hr] + [t for t, hb in zip(gb, has_b)
                                                                if hb]
        p = ctx.plan
        N.check(N.lib().hgnn_split_weight_grads_multi(
            len(ctx.metas), p.a_nrel, N.ptr_array(dws), N.ptr_array(dbs), p.a_ks, p.a_kroot,
            p.a_sc, ctx.h, N.ptr_array(dwl), N.ptr_array(dwr), N.ptr_array(dbl),
            N.stream_ptr(ctx.dev)), "hgnn_split_weight_grads_multi")
        return (None, *ret)


class _FuseMultiPlan:
    """The host arrays of one multi-update fuse (built once per set of parameter buffers)."""
    __slots__ = ("a_nrel", "a_wl", "a_wr", "a_bl", "a_ks", "a_sc", "a_kroot")

    def __init__(self, metas, groups):
        wl = [t for g in groups for t in g[0]]
        wr = [t for g in groups for t in g[1]]
        bl = [t for g in groups for t in g[2]]
        self.a_nrel = N.int_array([len(m[0]) for m in metas])
        self.a_wl, self.a_wr, self.a_bl = N.ptr_array(wl), N.ptr_array(wr), N.ptr_array(bl)
        self.a_ks = N.int_array([k for m in metas for k in m[0]])
        self.a_sc = N.float_array([x for m in metas for x in m[2]])
        self.a_kroot = N.int_array([m[1] for m in metas])


_FUSE_MULTI_PLANS: Dict[tuple, _FuseMultiPlan] = {}


def _fuse_multi_plan(metas, groups) -> _FuseMultiPlan:
    key = (metas, tuple(0 if t is None else t.data_ptr()
                        for g in groups for part in g for t in part))
    plan = _FUSE_MULTI_PLANS.get(key)
    if plan is None:
        if len(_FUSE_MULTI_PLANS) >= 1024:
            _FUSE_MULTI_PLANS.clear()
        plan = _FUSE_MULTI_PLANS[key] = _FuseMultiPlan(metas, groups)
    return plan


def fuse_weights_multi(groups) -> List[Tuple[torch.Tensor, Optional[torch.Tensor]]]:
    """``fuse_weights`` for several destination updates (``groups``: (wl, wr, bl, scales) each,
    one hidden width) in one launch each way; one update, or more than 4, falls back to the
    per-update calls."""
    if len(groups) == 1 or len(groups) > 4:
        return [fuse_weights(*g) for g in groups]
    metas, flat = [], []
    for wl, wr, bl, scales in groups:
        ks = tuple(int(t.shape[1]) for t in wl)
        roots = [t for t in wr if t is not None]
        metas.append((ks, int(roots[0].shape[1]) if roots else 0,
                      tuple(float(x) for x in scales), tuple(t is not None for t in wr),
                      tuple(t is not None for t in bl)))
        flat += [*wl, *roots, *[t for t in bl if t is not None]]
    flat = [t.contiguous() for t in flat]     # (parameters are; the plan keys on addresses)
    outs = iter(_FuseWeightsMulti.apply(tuple(metas), *flat))
    return [(next(outs), next(outs) if any(m[4]) else None) for m in metas]


# ----------------------------------------------------------------------------- layer spec
@dataclasses.dataclass(frozen=True)
class DstGroup:
    dst: str
    rels: Tuple[Tuple[str, RelationCSR], ...]   # (source type, relation structure)
    root: bool                                   # x_dst segment present (root_weight)
    relu: bool
    # per relation: project the SOURCE table first (lin_l(mean x_j) == mean(lin_l x_j), bias
    # kept in the destination update) — see use_pre_projection
    pre: Tuple[bool, ...] = ()
    # destinations = the first n_root rows of the dst type's table (a sampled block: the next
    # layer's nodes lead the current ones); None: the whole table
    n_root: Optional[int] = None
    # the root segment is the whole input ``root_src`` instead (a block whose relations gather
    # from the global tables: its destinations' own rows come as a separate input)
    root_src: Optional[str] = None


def _root_type(g: DstGroup) -> str:
    return g.dst if g.root_src is None else g.root_src


def _root(g: DstGroup, xs) -> torch.Tensor:
    """The destination rows' own features (the root segment): a prefix view in a block."""
    if g.root_src is not None:
        return xs[g.root_src]
    x = xs[g.dst]
    return x if g.n_root is None else x[:g.n_root]


def _root_grad_buffer(g: DstGroup, xs, gx, prefix=None) -> torch.Tensor:
    """Allocates gx[dst] and returns the view the root segment's dgrad writes (a block's prefix;
    the rows after it are zero until the K2s add into them — or, with ``prefix`` (a dict), left
    unwritten and recorded there: the first K2 round writes them fresh, ``_k2_rounds``)."""
    x = xs[_root_type(g)]
    if g.n_root is None or g.root_src is not None:
        gx[_root_type(g)] = torch.empty_like(x)
        return gx[_root_type(g)]
    if prefix is not None:
        gx[g.dst] = torch.empty_like(x)
        prefix[g.dst] = int(g.n_root)
    else:
        gx[g.dst] = torch.zeros_like(x)
    return gx[g.dst][:g.n_root]


PRE_PROJECTION = os.environ.get("HGNN_PREPROJECT", "1") == "1"


def use_pre_projection(x_src: torch.Tensor, x_dst: torch.Tensor, hidden: int,
                       root: bool) -> bool:
    """Whether a relation's lin_l should run on its source table before the mean gather.

    The mean is linear, so ``W (mean_j x_j) = mean_j (W x_j)``: projecting the N_src source rows
    and gathering the projected rows replaces the [N_dst x d_src] part of the destination
    projection by an [N_src x d_src] one.  Worth it when the source table is at most half the
    destination table (cfg4 layer 2: 1M posts -> 9M users halves the user-side K3 flops, forward
    and backward) and the gathered rows do not widen (d_src >= hidden).  Only where the backward
    needs the source gradient anyway (``x_src.requires_grad``) or there is no backward: the
    projection's weight gradient is dP^T x_src with dP = the mean scatter's transpose of dz, a
    K2 pass the aggregate-first order does not need when x_src is a static input (layer 1).
    Rounding differs from the reference's order only at the fp32 ulp level.  HGNN_PREPROJECT=0
    turns it off."""
    if not (PRE_PROJECTION and root):
        return False
    if 2 * x_src.shape[0] > x_dst.shape[0] or x_src.shape[1] < hidden:
        return False
    return bool(x_src.requires_grad or not torch.is_grad_enabled())


@dataclasses.dataclass(frozen=True)
class LayerSpec:
    types: Tuple[str, ...]                       # order of node-feature inputs
    groups: Tuple[DstGroup, ...]


class _Lanes:
    """Two in-order HIP streams (the caller's current stream + one side stream per device) for
    independent kernel chains.  Every tensor that escapes a side-stream chain is allocated on the
    main stream beforehand or record_stream()'d for it, and the main stream joins the side
    stream before returning, so the caching allocator never hands out memory still in use.
    Off by default: on cfg2 every overlapped pair slowed each other by as much as the overlap
    saved (layers: 10.55 vs 10.51 ms/step, the gathers already saturate the memory system; loss:
    the sort beside pass A stretched 0.49 -> 1.66 ms — pass A's workgroups hold every CU, so the
    sort's only get dispatched as it drains).  HGNN_STREAMS=1 turns it on."""

    _side: Dict[torch.device, torch.cuda.Stream] = {}
    enabled = os.environ.get("HGNN_STREAMS", "0") == "1"

    def __init__(self, dev: torch.device, n_chains: int, force: bool = False):
        self.main = self.side = None
        if (self.enabled or force) and n_chains > 1:
            self.main = torch.cuda.current_stream(dev)
            self.side = _Lanes._side.get(dev)
            if self.side is None:
                self.side = _Lanes._side[dev] = torch.cuda.Stream(dev)
            self.side.wait_stream(self.main)

    def ctx(self, i: int):
        """The stream context of chain i: a no-op with one lane (no Stream objects built — at a
        few hundred per sampled mini-batch step they were a visible share of its host time)."""
        if self.side is None:
            return contextlib.nullcontext()
        return torch.cuda.stream(self.side if i % 2 == 1 else self.main)

    def escape(self, i: int, *tensors):
        if self.side is not None and i % 2 == 1:
            for t in tensors:
                if t is not None:
                    t.record_stream(self.main)

    def join(self):
        if self.side is not None:
            self.main.wait_stream(self.side)


class _HeteroLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec: LayerSpec, *flat):
        nt = len(spec.types)
        xs = dict(zip(spec.types, flat[:nt]))
        wb = flat[nt:]
        ng = len(spec.groups)
        outs, aggrs_by_g, masks = [None] * ng, [None] * ng, [None] * ng
        dev = flat[0].device
        lanes = _Lanes(dev, ng)
        many = None
        if lanes.side is None and not any(any(g.pre) for g in spec.groups):
            # every relation's K1 of the layer in one launch (sampled blocks; gather_mean_many
            # falls back to one launch each where they do not qualify)
            many = iter(gather_mean_many([(xs[src], csr) for g in spec.groups
                                          for src, csr in g.rels]))
        if many is not None:
            # and every destination type's K3 in one native call (the split path's column blocks
            # one launch for both types, hgnn_linear_fwd_multi)
            jobs = []
            for gi, g in enumerate(spec.groups):
                w, b = wb[2 * gi], wb[2 * gi + 1]
                aggrs = [next(many) for _ in g.rels]
                segs = aggrs + ([_root(g, xs)] if g.root else [])
                mk = relu_mask_for(segs[0].shape[0], int(w.shape[0]), g.relu, dev,
                                   sum(int(t.shape[1]) for t in segs))
                jobs.append((segs, w.contiguous(), None if b is None else b.contiguous(), g.relu,
                             mk))
                aggrs_by_g[gi], masks[gi] = aggrs, mk
            outs = linear_fwd_many(jobs)
        for gi, g in enumerate(spec.groups if many is None else ()):   # independent chains
            w, b = wb[2 * gi], wb[2 * gi + 1]
            with lanes.ctx(gi):
                if any(g.pre):
                    # pre-projected relations: P = x_src W_r^T, gathered (means summed into
                    # one [N_dst, h] input) and added in the destination update's epilogue
                    cols = _group_columns(g, xs)
                    add, aggrs = None, []
                    for (src, csr), pre, (o, k) in zip(g.rels, g.pre, cols):
                        if pre:
                            P = linear_fwd([xs[src]], w[:, o:o + k].contiguous(), None, False)
                            add = gather_mean(P, csr, out=add)
                            del P
                        else:
                            aggrs.append(gather_mean(xs[src], csr))
                    segs = aggrs + ([_root(g, xs)] if g.root else [])
                    mk = relu_mask_for(_root(g, xs).shape[0], int(w.shape[0]), g.relu, dev,
                                       sum(int(t.shape[1]) for t in segs))
                    y = linear_fwd(segs, _main_weight(g, w, cols),
                                   None if b is None else b.contiguous(), g.relu, add=add,
                                   mask_out=mk)
                    del add
                else:
                    aggrs = [gather_mean(xs[src], csr) for src, csr in g.rels]
                    segs = aggrs + ([_root(g, xs)] if g.root else [])
                    mk = relu_mask_for(segs[0].shape[0], int(w.shape[0]), g.relu, dev,
                                       sum(int(t.shape[1]) for t in segs))
                    y = linear_fwd(segs, w.contiguous(), None if b is None else b.contiguous(),
                                   g.relu, mask_out=mk)
            lanes.escape(gi, y, mk, *aggrs)
            outs[gi], aggrs_by_g[gi], masks[gi] = y, aggrs, mk
        lanes.join()
        aggrs_all = [a for aggrs in aggrs_by_g for a in aggrs]
        ctx.spec = spec
        ctx.masks = masks          # ReLU bits of each output (None where there is no bit form)
        ctx.has_b = [b is not None for b in wb[1::2]]
        ctx.save_for_backward(*flat[:nt], *[t for t in wb if t is not None], *aggrs_all, *outs)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        spec: LayerSpec = ctx.spec
        nt, ng = len(spec.types), len(spec.groups)
        saved = list(ctx.saved_tensors)
        xs = dict(zip(spec.types, saved[:nt]))
        pos = nt
        wbs = []
        for hb in ctx.has_b:
            w = saved[pos]; pos += 1
            b = None
            if hb:
                b = saved[pos]; pos += 1
            wbs.append((w, b))
        aggrs_all = saved[pos:pos + sum(_n_main_rels(g) for g in spec.groups)]
        pos += len(aggrs_all)
        outs = saved[pos:pos + ng]
        need = ctx.needs_input_grad[1:]
        need_x = dict(zip(spec.types, need[:nt]))
        gx: Dict[str, Optional[torch.Tensor]] = {t: None for t in spec.types}
        gwb: List[Optional[torch.Tensor]] = [None] * (2 * ng)
        pending: Dict[str, list] = {}   # target type -> [(dA, csr)] for K2, after the roots
        # phase 1: every destination type's K3 backward (independent chains); all outputs
        # allocated here on the main stream
        jobs = []
        ai = 0
        pre_jobs = []
        # sampled blocks on one lane: a destination type that K2s will write (its relations'
        # sources) gets its block gradient unzeroed, the first K2 round writing past the prefix
        one_lane = (_Lanes(saved[0].device, 2).side is None
                    and not any(any(g.pre) for g in spec.groups))
        k2_targets = {src for g in spec.groups for src, csr in g.rels
                      if need_x[src] and csr.num_edges > 0}
        prefix: Dict[str, int] = {}
        for gi, g in enumerate(spec.groups):
            aggrs = aggrs_all[ai:ai + _n_main_rels(g)]
            ai += _n_main_rels(g)
            dout = douts[gi]
            w, b = wbs[gi]
            need_w, need_b = need[nt + 2 * gi], (b is not None and need[nt + 2 * gi + 1])
            if dout is None:
                continue
            if any(g.pre):
                pre_jobs.append((gi, g, aggrs, w, dout.contiguous(), need_w, need_b,
                                 ctx.masks[gi]))
                continue
            dxs: List[Optional[torch.Tensor]] = []
            for (src, csr), a in zip(g.rels, aggrs):
                if need_x[src] and csr.num_edges > 0:
                    dA = torch.empty_like(a)
                    dxs.append(dA)
                    pending.setdefault(src, []).append((dA, csr))
                else:
                    dxs.append(None)
            segs = list(aggrs)
            if g.root:
                segs.append(_root(g, xs))
                fresh = one_lane and _root_type(g) in k2_targets
                dxs.append(_root_grad_buffer(g, xs, gx, prefix if fresh else None)
                           if need_x[_root_type(g)] else None)
            jobs.append((gi, g, segs, w, dout.contiguous(), dxs, need_w, need_b))
        lanes = _Lanes(saved[0].device, len(jobs))
        if one_lane and lanes.side is None:
            # one native call for the destination types' K3 backward (hgnn_linear_bwd_multi)
            res = linear_bwd_many([(segs, w, dout, outs[gi] if g.relu else None, dxs, need_w,
                                    need_b, ctx.masks[gi])
                                   for gi, g, segs, w, dout, dxs, need_w, need_b in jobs])
            for (gi, *_), (dw, db) in zip(jobs, res):
                gwb[2 * gi], gwb[2 * gi + 1] = dw, db
            jobs = []
        for li, (gi, g, segs, w, dout, dxs, need_w, need_b) in enumerate(jobs):
            with lanes.ctx(li):
                dw, db = linear_bwd(segs, w, dout, outs[gi] if g.relu else None, dxs, need_w,
                                    need_b, mask=ctx.masks[gi])
            lanes.escape(li, dw, db)
            gwb[2 * gi], gwb[2 * gi + 1] = dw, db
        lanes.join()
        # groups with pre-projected relations (main stream): dz once, the destination update's
        # backward on it, then per pre-projected relation the K2 of dz into the projected source
        # rows and the projection's backward
        for gi, g, aggrs, w, dout, need_w, need_b, mk in pre_jobs:
            gwb[2 * gi], gwb[2 * gi + 1] = _pre_group_backward(
                g, xs, aggrs, w, dout, outs[gi], need_x, need_w, need_b, gx, pending, mk)
        # phase 2: K2 per target type (different targets are independent chains)
        for t in pending:
            if gx[t] is None:
                gx[t] = torch.zeros_like(xs[t])
        lanes = _Lanes(saved[0].device, len(pending))
        if lanes.side is None and len(pending) > 1 and _k2_rounds(pending, gx, prefix):
            return (None, *[gx[t] for t in spec.types], *gwb)
        for t, n in prefix.items():          # (no rounds after all: zero what K2s add into)
            gx[t][n:].zero_()
        for li, (t, items) in enumerate(pending.items()):
            with lanes.ctx(li):
                for dA, csr in items:
                    scatter_mean_bwd(dA, csr, out=gx[t])
        lanes.join()
        return (None, *[gx[t] for t in spec.types], *gwb)


def _k2_rounds(pending, gx, prefix=None) -> bool:
    """The K2s of a layer's backward as rounds of one launch each: round r takes the r-th
    relation of every target type (distinct outputs, so no two jobs of a launch add into the
    same rows; each target's relations keep their order).  ``prefix[t]``: gx[t] holds only its
    first rows (the root term); round 0 adds into those and writes the rest fresh.  False
    (nothing launched) where the relations do not qualify (source-blocked or heavy-row gathers,
    ``_multi_ok``)."""
    prefix = prefix or {}
    jobs_by_round: List[list] = []
    for t, items in pending.items():
        for r, (dA, csr) in enumerate(items):
            if csr.num_edges and gather_blocks(dA, csr.num_edges) > 1:
                return False
            if len(jobs_by_round) <= r:
                jobs_by_round.append([])
            jobs_by_round[r].append((dA.contiguous(), csr, gx[t]))
    for jobs in jobs_by_round:
        if len(jobs) > 1 and not _multi_ok([(dA, csr.bwd, o) for dA, csr, o in jobs]):
            return False
    if any(len(j) == 1 for j in jobs_by_round[:1]) and prefix:
        return False                         # round 0 must be a multi launch to honour prefix
    targets = list(pending)
    for r, jobs in enumerate(jobs_by_round):
        if len(jobs) == 1:
            dA, csr, o = jobs[0]
            scatter_mean_bwd(dA, csr, out=o)
        else:
            lim = None
            if r == 0 and prefix:
                lim = [prefix.get(t, 0) for t in targets if pending[t]]
            _gather_multi([(dA, csr.bwd, o) for dA, csr, o in jobs], mean=False,
                          accumulate=True, edge_ws=[csr.bwd_weights for _, csr, _ in jobs],
                          acc_limit=lim)
    return True


def _group_columns(g: DstGroup, xs) -> List[Tuple[int, int]]:
    """(offset, width) of each relation's lin_l block in the group's fused weight."""
    cols, o = [], 0
    for src, _ in g.rels:
        k = int(xs[src].shape[1])
        cols.append((o, k))
        o += k
    return cols


def _n_main_rels(g: DstGroup) -> int:
    return sum(1 for i in range(len(g.rels)) if not (g.pre and g.pre[i]))


def _main_weight(g: DstGroup, w: torch.Tensor, cols) -> torch.Tensor:
    """The fused weight without the pre-projected relations' lin_l blocks."""
    keep = [w[:, o:o + k] for (o, k), pre in zip(cols, g.pre) if not pre]
    if g.root:
        keep.append(w[:, cols[-1][0] + cols[-1][1]:] if cols else w)
    return torch.cat(keep, dim=1).contiguous()


def relu_grad(dout: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """dz = dout * (out > 0): ReLU's backward from its output (one streaming pass)."""
    dz = torch.empty_like(dout)
    n = dout.numel()
    with _timed("relu_grad", 12 * n):
        N.check(N.lib().hgnn_hetero_epilogue_bwd(1, N.float_array([1.0]), n, 1, N.ptr(out),
                                                 N.ptr(dout), N.ptr_array([dz]),
                                                 N.stream_ptr(dout.device)),
                "hgnn_hetero_epilogue_bwd")
    return dz


def _pre_group_backward(g: DstGroup, xs, aggrs, w, dout, y, need_x, need_w, need_b, gx,
                        pending, mask=None):
    """Backward of a destination group with pre-projected relations: returns (dW, db) in the
    fused weight's column layout; source gradients go to ``gx`` / ``pending`` (K2 list)."""
    cols = _group_columns(g, xs)
    # the destination update's backward over the remaining segments also writes the masked dz
    # that the pre-projected relations' K2 scatters (from the pass that masks it anyway)
    dz = torch.empty_like(dout) if g.relu else dout
    segs, seg_cols, dxs = [], [], []
    ai = 0
    for (src, csr), pre, c in zip(g.rels, g.pre, cols):
        if pre:
            continue
        a = aggrs[ai]
        ai += 1
        segs.append(a)
        seg_cols.append(c)
        if need_x[src] and csr.num_edges > 0:
            dA = torch.empty_like(a)
            dxs.append(dA)
            pending.setdefault(src, []).append((dA, csr))
        else:
            dxs.append(None)
    dx_add = [False] * len(dxs)
    if g.root:
        segs.append(_root(g, xs))
        o = cols[-1][0] + cols[-1][1] if cols else 0
        seg_cols.append((o, int(w.shape[1]) - o))
        if need_x[g.dst]:
            # the root gradient is added into the destination table's gradient in the dgrad pass
            # when another update already wrote it (no separate add); else it is that gradient
            # (a block's prefix of a zeroed table: its other rows wait for the K2s)
            dx_add.append(gx[g.dst] is not None)
            if gx[g.dst] is None:
                gx[g.dst] = (torch.empty_like(xs[g.dst]) if g.n_root is None
                             else torch.zeros_like(xs[g.dst]))
            dxs.append(gx[g.dst] if g.n_root is None else gx[g.dst][:g.n_root])
        else:
            dxs.append(None)
            dx_add.append(False)
    dw = torch.empty_like(w) if need_w else None
    dw_main, db = linear_bwd(segs, _main_weight(g, w, cols), dout, y if g.relu else None, dxs,
                             need_w, need_b, dz_out=dz if g.relu else None, mask=mask,
                             dx_add=dx_add)
    if dw is not None:
        o = 0
        for (co, k) in seg_cols:
            dw[:, co:co + k].copy_(dw_main[:, o:o + k])
            o += k
    # pre-projected relations: dP = K2(dz) over the CSC, then P = x_src W_r^T's backward
    for (src, csr), pre, (o, k) in zip(g.rels, g.pre, cols):
        if not pre:
            continue
        x_src = xs[src]
        dP = scatter_mean_bwd(dz, csr)
        add = need_x[src] and gx[src] is not None   # added into the table's gradient in place
        dxp = (gx[src] if add else torch.empty_like(x_src)) if need_x[src] else None
        dwp, _ = linear_bwd([x_src], w[:, o:o + k].contiguous(), dP, None, [dxp], need_w, False,
                            dx_add=[add])
        if dw is not None:
            dw[:, o:o + k].copy_(dwp)
        if dxp is not None:
            gx[src] = dxp
    return dw, db


def hetero_layer(spec: LayerSpec, x_dict: Dict[str, torch.Tensor],
                 weights: Sequence[Tuple[torch.Tensor, Optional[torch.Tensor]]]
                 ) -> Dict[str, torch.Tensor]:
    flat: List[Optional[torch.Tensor]] = [x_dict[t] for t in spec.types]
    for w, b in weights:
        flat.extend([w, b])
    N.require_device(*[t for t in flat if t is not None])
    for t in flat[:len(spec.types)]:
        _check_f32(t, "node features")
    for g in spec.groups:
        if g.root_src is not None:
            if any(g.pre) or g.n_root is not None or not g.root:
                raise ValueError("hetero_layer: root_src takes a root segment, no n_root and no "
                                 "pre-projected relation")
            n = int(x_dict[g.root_src].shape[0])
        else:
            n = int(x_dict[g.dst].shape[0]) if g.n_root is None else int(g.n_root)
        for src, csr in g.rels:
            if csr.n_dst != n or csr.n_src != int(x_dict[src].shape[0]):
                raise ValueError(f"hetero_layer: relation {src}->{g.dst} is {csr.n_src}->"
                                 f"{csr.n_dst} rows, the tables give {x_dict[src].shape[0]}->{n}")
    outs = _HeteroLayer.apply(spec, *flat)
    return {g.dst: y for g, y in zip(spec.groups, outs)}


# ----------------------------------------------------------------------------- link loss
def link_loss(user_emb: torch.Tensor, post_emb: torch.Tensor, pos_edges: torch.Tensor,
              neg_p: torch.Tensor, pos_weights: torch.Tensor) -> torch.Tensor:
    """The reference training loss (train_gnn.py:259-281), on the device with torch ops.

    ``BCEWithLogitsLoss()`` has mean reduction, so ``(pos_weights * pos_loss).mean()`` equals
    ``mean(pos_weights) * pos_loss`` — reproduced as written."""
    pos_u, pos_p = pos_edges[0], pos_edges[1]
    u = user_emb[pos_u]
    pos_scores = (u * post_emb[pos_p]).sum(dim=1)
    neg_scores = (u * post_emb[neg_p]).sum(dim=1)
    crit = torch.nn.functional.binary_cross_entropy_with_logits
    pos_loss = crit(pos_scores, torch.ones_like(pos_scores))
    neg_loss = crit(neg_scores, torch.zeros_like(neg_scores))
    return (pos_weights * pos_loss).mean() + neg_loss


# ----------------------------------------------------------------------------- fused link loss
def _user_of_pos(csr: RelationCSR) -> torch.Tensor:
    """Static per graph: the user owning each position of the user-grouped CSC (int32)."""
    m = getattr(csr, "_uop", None)
    if m is None:
        rp = csr.bwd.rowptr
        deg = (rp[1:] - rp[:-1]).long()
        m = torch.repeat_interleave(torch.arange(csr.n_src, dtype=torch.int32, device=rp.device),
                                    deg).contiguous()
        csr._uop = m
    return m


def negatives_in_user_order(csr: RelationCSR, neg_p: torch.Tensor) -> torch.Tensor:
    """Re-order negatives drawn per COO edge (train_gnn.py:272) to the user-grouped order the
    fused kernel walks."""
    return neg_p.to(torch.int64)[csr.bwd.perm.long()].contiguous()


def _row_range(grouped, lo: int, hi: int):
    """Rows [lo, hi) of a grouping as a grouping of their own (rowptr slice with absolute offsets
    into the shared col), with its own skew plan — built once and cached on the grouping."""
    from .graph import GroupedEdges, _plan
    cache = grouped.__dict__.setdefault("_ranges", {})
    g = cache.get((lo, hi))
    if g is None:
        rp = grouped.rowptr[lo:hi + 1]
        g = cache[(lo, hi)] = GroupedEdges(rp, grouped.col, None, _plan(rp, hi - lo,
                                                                         grouped.plan.chunk),
                                           hi - lo)
    return g


def _sort_negatives(csr, neg_u_order, draw, neg, neg32: bool, uop, E: int, np_: int, err,
                    dev):
    """The negatives (user-grouped order) grouped by post: (rowptr over posts, users in that
    order), stable — the order the dP gather sums them in."""
    lib = N.lib()
    rowptr_n = torch.empty(np_ + 1, dtype=torch.int32, device=dev)
    nu_s = torch.empty(E, dtype=torch.int32, device=dev)
    ws = N.workspace(lib.hgnn_sort_pairs_ws_bytes(E, np_), dev)
    if draw is not None:
        # draws computed in the sort's first pass (and again in the scoring pass: no
        # position-order copy is written)
        with _timed("sort_negatives", 4 * E * (2 * 4)):
            N.check(lib.hgnn_draw_sort_negatives(
                N.ptr(draw.seed), N.ptr(uop), E, np_, None, N.ptr(rowptr_n),
                N.ptr(nu_s), N.ptr(ws), ws.numel(), N.stream_ptr(dev)),
                "hgnn_draw_sort_negatives")
    elif neg32:
        # int32 keys: no validation pass (the scoring pass below counts out-of-range
        # negatives; the sort only misplaces such a key, never dereferences it)
        with _timed("sort_negatives", 4 * E * (2 * 4) + 4 * E):
            N.check(lib.hgnn_sort_pairs_i32(
                N.ptr(neg), N.ptr(uop), None, E, np_, N.ptr(rowptr_n), N.ptr(nu_s),
                None, None, N.ptr(ws), ws.numel(), N.stream_ptr(dev)),
                "hgnn_sort_pairs_i32")
    else:
        with _timed("sort_negatives", 4 * E * (2 + 1 + 4) + 4 * E):
            N.check(lib.hgnn_sort_pairs_i64(
                N.ptr(neg), N.ptr(uop), None, E, np_, N.ptr(rowptr_n), N.ptr(nu_s),
                None, N.ptr(err[1:]), N.ptr(ws), ws.numel(), N.stream_ptr(dev)),
                "hgnn_sort_pairs_i64")
    return rowptr_n, nu_s


class PresortedNegatives:
    """The loss's negatives already grouped by post (``presort_negatives``): the sharded step
    sorts them under a collective, ahead of the loss that consumes them.  It holds the grouping
    and the draws it was made from (the objects themselves, compared with ``is``: an id could be
    reused by a new object once the old one is freed), so a loss over other edges or other
    draws is refused."""

    def __init__(self, csr, neg_p, neg_order: str, n_posts: int, rowptr, users):
        self.csr, self.neg_p, self.neg_order = csr, neg_p, neg_order
        self.n_posts = int(n_posts)
        self.rowptr, self.users = rowptr, users

    def check_draws(self, neg_p, neg_order: str, where: str) -> None:
        if neg_order != self.neg_order:
            raise ValueError(f"{where}: presorted negatives were grouped with neg_order="
                             f"{self.neg_order!r}, the loss got neg_order={neg_order!r}")
        if neg_p is not self.neg_p:
            raise ValueError(f"{where}: presorted negatives of other draws")

    def check_edges(self, csr, n_posts: int) -> None:
        if csr is not self.csr or int(n_posts) != self.n_posts:
            raise ValueError("edge_bce_loss: the presorted negatives are for other edges")


def _neg_inputs(neg_u_order):
    draw = neg_u_order if isinstance(neg_u_order, NegativeDraw) else None
    neg32 = neg_u_order.dtype == torch.int32
    if draw is not None:
        neg = None
    else:
        neg = neg_u_order.contiguous() if neg32 else neg_u_order.to(torch.int64).contiguous()
    return draw, neg32, neg


def presort_negatives(n_users: int, n_posts: int, pos_edges: torch.Tensor, neg_p,
                      neg_order: str) -> PresortedNegatives:
    """The grouping ``edge_bce_loss_raw`` would sort its negatives into, done now (it needs
    only the edges and the draws, not the embeddings); pass it back as ``presorted=`` with the
    same ``neg_p`` and ``neg_order`` (required here: the two loss entry points default to
    different orders)."""
    csr = relation_csr_for_loss(pos_edges, n_users, n_posts)
    neg_u = _negatives_user_order(csr, neg_p, neg_order)
    draw, neg32, neg = _neg_inputs(neg_u)
    dev = csr.fwd.rowptr.device
    err = torch.zeros(2, dtype=torch.int32, device=dev)
    E = csr.num_edges
    rp, us = _sort_negatives(csr, neg_u, draw, neg, neg32, _user_of_pos(csr), E, n_posts, err,
                             dev)
    return PresortedNegatives(csr, neg_p, neg_order, n_posts, rp, us)


def _edge_bce(U, P, csr: RelationCSR, neg_u_order, cscale, check: bool, n_total: int,
              ready=None, on_dP=None, p_chunks=None, presorted=None):
    """Loss value and its gradients for a unit upstream gradient: (loss, dU, dP).  ``on_dP(dP)``,
    if given, is called once dP's kernels are enqueued and before the scoring pass (dU, the loss)
    is: the sharded step starts dP's reduce-scatter there, under the scoring pass.
    ``p_chunks`` (the sharded step): [(lo, hi, ready_fn)] — the post table arrives in row blocks
    (parallel.DistEnv.broadcast_slices_async); dP's rows [lo, hi) need only those rows of P, so
    the dP gather runs block by block as each lands (ready_fn: a stream wait), and the scoring
    pass, which reads all of P, after the last."""
    U = _check_f32(U, "edge_bce_loss user_emb")
    P = _check_f32(P, "edge_bce_loss post_emb")
    draw = neg_u_order if isinstance(neg_u_order, NegativeDraw) else None
    dev = N.require_device(U, P, draw.seed if draw is not None else neg_u_order)
    lib, s = N.lib(), N.stream_ptr(dev)
    nu, np_, d, E = U.shape[0], P.shape[0], int(U.shape[1]), csr.num_edges
    if P.shape[1] != d or nu != csr.n_src or np_ != csr.n_dst:
        raise ValueError("edge_bce_loss: embedding shapes do not match the positive edges")
    if E == 0:
        # a shard without positive edges (parallel.py): its share of the loss and gradients is
        # zero, and no kernel would read a negative (the C ABI rejects the empty tensor's null
        # pointer whenever the global edge count is non-zero)
        if ready is not None:
            ready()
        return (torch.zeros((), dtype=torch.float32, device=dev), torch.zeros_like(U),
                torch.zeros_like(P))
    ub, pf = csr.bwd, csr.fwd
    dU = torch.empty_like(U)
    part = torch.empty(int(lib.hgnn_edge_score_parts(nu)), dtype=torch.float32, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    # err[0]: zeroed and counted by the scoring pass, err[1] by the int64 negatives sort
    err = torch.empty(2, dtype=torch.int32, device=dev)
    c = cscale.to(torch.float32).reshape(()).contiguous()
    inv_e = 1.0 / n_total if n_total > 0 else 0.0
    uop = _user_of_pos(csr)
    neg32 = neg_u_order.dtype == torch.int32          # sample_negatives' / draw_negatives' draws
    if draw is not None:
        if draw.n != E or draw.num_posts != np_:
            raise ValueError("edge_bce_loss: the NegativeDraw does not match the positive edges")
        neg = None   # drawn again where read (the sort's first pass, the scoring pass)
    else:
        neg = neg_u_order.contiguous() if neg32 else neg_u_order.to(torch.int64).contiguous()
    dP = torch.empty_like(P)
    # dP chain (side stream under HGNN_STREAMS=1): sort the negatives (post, user) by post,
    # then the two dP gathers, each edge's weight recomputed from <U[u], P[post]>
    # (hgnn_score_gather); pass A (loss + dU) needs none of it.
    lanes = _Lanes(dev, 2)
    with lanes.ctx(1):
        if presorted is not None:
            presorted.check_edges(csr, np_)
            rowptr_n, nu_s = presorted.rowptr, presorted.users
        else:
            rowptr_n, nu_s = _sort_negatives(csr, neg_u_order, draw, neg, neg32, uop, E, np_,
                                             err, dev)
    if ready is not None and p_chunks is None:
        # P is still arriving (parallel.py's all-gather of the post table): the sort above
        # needs only the edges, so it ran ahead; every kernel below reads P
        ready()
        if lanes.side is not None:
            lanes.side.wait_stream(lanes.main)
    with lanes.ctx(1):
        from .graph import NO_SPLIT, GroupedEdges, Plan
        negs = GroupedEdges(rowptr_n, nu_s, nu_s, Plan(NO_SPLIT, 0, 0, None, None), np_)
        if p_chunks is not None:
            for lo, hi, rdy in p_chunks:
                if rdy is not None:
                    rdy()
                if hi > lo:
                    ng = GroupedEdges(rowptr_n[lo:hi + 1], nu_s, None,
                                      Plan(NO_SPLIT, 0, 0, None, None), hi - lo)
                    _score_gather2(U, P[lo:hi], _row_range(pf, lo, hi), ng, c, inv_e, dP[lo:hi])
        else:
            # (Measured and not kept, round 5: this gather in 8 source-block passes like K1,
            # 32.83 vs 31.32 ms at cfg4 — each pass re-reads its rows' P vectors and dP.)
            _score_gather2(U, P, pf, negs, c, inv_e, dP)
        if on_dP is not None:
            on_dP(dP)
    if ready is not None and p_chunks is not None:
        ready()                                 # all of P, for the scoring pass
    with _timed(f"edge_score_d{d}", 4 * E * (2 * d + 1 + 2) + 8 * nu * d):
        if draw is not None:
            N.check(lib.hgnn_edge_score_fwd_draw(
                N.ptr(U), N.ptr(P), d, nu, np_, N.ptr(ub.rowptr), N.ptr(ub.col),
                N.ptr(draw.seed), n_total, N.ptr(c), N.ptr(dU), N.ptr(part), N.ptr(loss),
                N.ptr(err if check else None), s), "hgnn_edge_score_fwd_draw")
        elif neg32:
            N.check(lib.hgnn_edge_score_fwd_i32(
                N.ptr(U), N.ptr(P), d, nu, np_, N.ptr(ub.rowptr), N.ptr(ub.col),
                N.ptr(neg), n_total, N.ptr(c), N.ptr(dU), N.ptr(part), N.ptr(loss),
                N.ptr(err if check else None), s), "hgnn_edge_score_fwd_i32")
        else:
            N.check(lib.hgnn_edge_score_fwd(
                N.ptr(U), N.ptr(P), d, nu, np_, N.ptr(ub.rowptr), N.ptr(ub.col),
                N.ptr(neg), None, n_total, N.ptr(c), N.ptr(dU), None, None, None, None,
                N.ptr(part), N.ptr(loss), N.ptr(err if check else None), s),
                "hgnn_edge_score_fwd")
    lanes.join()
    if check and int(err[0]):
        raise ValueError("edge_bce_loss: negative post id out of range")
    return loss, dU, dP


class _EdgeBCELoss(torch.autograd.Function):
    """The forward computes dL/dU and dL/dP with the loss (one scoring pass, one dP gather) and
    keeps them; the first backward scales them in place by the upstream gradient and hands them
    on (no copy: 2 x 4.6 GB at cfg4).  A second backward through a retained graph
    (``retain_graph=True``) recomputes them from the saved embeddings and the same negatives —
    the kernels are deterministic, so it returns what the first did, as torch's loss would.
    For that recompute U and P stay saved until the graph is freed (as torch's own loss saves
    its inputs): at cfg4 4.6 + 0.5 GB of the 288 GB, held from the forward to the end of the
    backward, which the split K3 backward (mask bits, not the outputs) would otherwise release
    after this loss's backward."""

    @staticmethod
    def forward(ctx, U, P, csr: RelationCSR, neg_u_order, cscale, check: bool, n_total: int,
                ready=None, presorted=None):
        loss, dU, dP = _edge_bce(U, P, csr, neg_u_order, cscale, check, n_total, ready,
                                 presorted=presorted)
        ctx.grads = (dU, dP)
        ctx.save_for_backward(U, P)
        ctx.args = (csr, neg_u_order, cscale, n_total)
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, go):
        if ctx.grads is None:        # retained graph, second backward: recompute
            U, P = ctx.saved_tensors
            csr, neg_u_order, cscale, n_total = ctx.args
            _, dU, dP = _edge_bce(U, P, csr, neg_u_order, cscale, False, n_total)
        else:
            dU, dP = ctx.grads
            ctx.grads = None         # handed on: autograd may accumulate into them from here
        if not getattr(go, UNIT_GRAD, False):
            g = go.to(torch.float32).reshape(()).contiguous()
            lib, s = N.lib(), N.stream_ptr(dU.device)
            for t in (dU, dP):   # in place; a no-op launch for loss.backward()'s gradient of 1
                N.check(lib.hgnn_scale_unless_one(N.ptr(t), t.numel(), N.ptr(g), s),
                        "hgnn_scale_unless_one")
        return dU, dP, None, None, None, None, None, None, None


# A tensor carrying this attribute (set True) is a gradient of exactly 1 that nobody writes:
# ``loss.backward(unit)`` with it skips the loss's scaling launches (minibatch.CapturedStep).
UNIT_GRAD = "_hgnn_unit_grad"


def unit_grad(device) -> torch.Tensor:
    """A scalar 1.0 marked ``UNIT_GRAD``, for ``loss.backward(unit)``: the fused loss then hands
    on its gradients unscaled, with no launch (the implicit ``loss.backward()`` makes a fill
    and, per gradient, a scale-by-1 launch — three graph nodes of a captured step)."""
    t = torch.ones((), dtype=torch.float32, device=device)
    setattr(t, UNIT_GRAD, True)
    return t


def edge_bce_loss(user_emb: torch.Tensor, post_emb: torch.Tensor, pos_edges: torch.Tensor,
                  neg_p: torch.Tensor, pos_weights: Optional[torch.Tensor],
                  neg_order: str = "edge", check: bool = True,
                  n_edges_total: Optional[int] = None,
                  cscale: Optional[torch.Tensor] = None, ready=None,
                  presorted: Optional["PresortedNegatives"] = None) -> torch.Tensor:
    """Fused HIP version of :func:`link_loss` (same value, same gradients).

    ``neg_order='edge'``: ``neg_p[e]`` is the negative of COO edge e (the reference's layout);
    ``'user'``: already in the user-grouped order (what :func:`sample_negatives` draws).
    ``check`` costs one host sync (the reference syncs every step with ``loss.item()``).
    ``n_edges_total`` / ``cscale`` (= mean of ALL pos_weights) let a shard of the positive edges
    produce its additive share of the global loss (parallel.py); ``ready()``, if given, is
    called once the negatives sort is enqueued and before any kernel reads ``post_emb`` (the
    sharded path's post-table all-gather finishes under the sort).  ``presorted``: the grouping
    of these negatives from :func:`presort_negatives`, done ahead (e.g. on a side stream under the
    forward; the caller orders the streams)."""
    csr = relation_csr_for_loss(pos_edges, user_emb.shape[0], post_emb.shape[0])
    if neg_p.shape[0] != csr.num_edges:
        raise ValueError("one negative per positive edge is required (train_gnn.py:272)")
    neg_u = _negatives_user_order(csr, neg_p, neg_order)
    if cscale is None:
        cscale = pos_weights.to(torch.float32).mean()
    n_total = csr.num_edges if n_edges_total is None else int(n_edges_total)
    if presorted is not None:
        presorted.check_draws(neg_p, neg_order, "edge_bce_loss")
    return _EdgeBCELoss.apply(user_emb, post_emb, csr, neg_u, cscale, check, n_total, ready,
                              presorted)


def edge_bce_loss_raw(user_emb: torch.Tensor, post_emb: torch.Tensor, pos_edges: torch.Tensor,
                      neg_p: torch.Tensor, n_edges_total: int, cscale: torch.Tensor,
                      neg_order: str = "user", ready=None, on_dP=None, p_chunks=None,
                      presorted: Optional[PresortedNegatives] = None):
    """:func:`edge_bce_loss` outside autograd: (loss, dL/dU, dL/dP) from the same kernels, for
    callers that run their own backward schedule (``parallel.UserShard.step``; ``on_dP``,
    ``p_chunks``: see ``_edge_bce``; ``presorted``: from :func:`presort_negatives` on the same
    edges and draws)."""
    csr = relation_csr_for_loss(pos_edges, user_emb.shape[0], post_emb.shape[0])
    neg_u = _negatives_user_order(csr, neg_p, neg_order)
    if presorted is not None:
        presorted.check_draws(neg_p, neg_order, "edge_bce_loss_raw")
    return _edge_bce(user_emb, post_emb, csr, neg_u, cscale, False, int(n_edges_total), ready,
                     on_dP, p_chunks, presorted)


def _negatives_user_order(csr, neg_p, neg_order):
    if isinstance(neg_p, NegativeDraw):
        if neg_order != "user":
            raise ValueError("a NegativeDraw is drawn in the user-grouped order (neg_order='user')")
        return neg_p
    return negatives_in_user_order(csr, neg_p) if neg_order == "edge" else neg_p.contiguous()


def relation_csr_for_loss(pos_edges, n_users, n_posts) -> RelationCSR:
    from .graph import relation_csr
    return relation_csr(pos_edges, n_users, n_posts)


class NegativeDraw:
    """One uniform negative post per positive edge, not yet materialised: the device seed of a
    counter-based draw (:func:`draw_negatives`).  The fused loss draws and groups them by post in
    one call (``hgnn_draw_sort_negatives``: the draws are computed inside the sort's first pass,
    not written by one kernel and read back by two); :meth:`tensor` gives the same int32 values
    as :func:`sample_negatives` would for the same seed."""

    def __init__(self, seed: torch.Tensor, n: int, num_posts: int):
        self.seed, self.n, self.num_posts = seed, int(n), int(num_posts)
        self.shape = (self.n,)
        self.dtype = torch.int32
        self.device = seed.device

    def tensor(self) -> torch.Tensor:
        out = torch.empty(self.n, dtype=torch.int32, device=self.device)
        if self.n:
            N.check(N.lib().hgnn_uniform_i32(N.ptr(self.seed), self.n, self.num_posts, N.ptr(out),
                                             N.stream_ptr(self.device)), "hgnn_uniform_i32")
        return out


def draw_negatives(pos_edges: torch.Tensor, num_posts: int,
                   generator: Optional[torch.Generator] = None) -> NegativeDraw:
    """:func:`sample_negatives` without the materialised array: the seed only (one tiny device
    draw from ``generator``, no host sync).  ``edge_bce_loss(..., neg_order='user')`` takes it."""
    dev = N.require_device(pos_edges)
    if num_posts < 1 or num_posts >= 2**31:
        raise ValueError(f"num_posts={num_posts} out of range")
    seed = torch.randint(0, 2**62, (1,), device=dev, dtype=torch.int64, generator=generator)
    return NegativeDraw(seed, int(pos_edges.shape[1]), num_posts)


def sample_negatives(pos_edges: torch.Tensor, num_posts: int,
                     generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """One uniform negative post per positive edge (train_gnn.py:272's ``torch.randint``), drawn
    directly in the user-grouped order: the draws are iid, so only their labels move.

    int32 draws from ``hgnn_uniform_i32`` (a counter-based generator seeded from ``generator``
    on the device, no host sync): in range by construction, so the loss sorts them without the
    int64 validation pass.  ``edge_bce_loss`` also takes int64 ``torch.randint`` negatives."""
    dev = N.require_device(pos_edges)
    E = int(pos_edges.shape[1])
    out = torch.empty(E, dtype=torch.int32, device=dev)
    if E == 0:
        return out
    if num_posts < 1 or num_posts >= 2**31:
        raise ValueError(f"num_posts={num_posts} out of range")
    seed = torch.randint(0, 2**62, (1,), device=dev, dtype=torch.int64,
                         generator=generator)
    N.check(N.lib().hgnn_uniform_i32(N.ptr(seed), E, int(num_posts), N.ptr(out),
                                     N.stream_ptr(dev)), "hgnn_uniform_i32")
    return out


# ----------------------------------------------------------------------------- composable ops
# Differentiable single-kernel ops, used where a fused layer does not apply (the partitioned
# multi-GPU path in parallel.py composes them around RCCL collectives).
class _GatherMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_src, csr: RelationCSR):
        ctx.csr = csr
        return gather_mean(x_src, csr)

    @staticmethod
    def backward(ctx, g):
        await_pending(g)     # the halo exchange's adjoint may still be in flight (parallel.py)
        if not ctx.needs_input_grad[0]:
            return None, None
        if ctx.csr.num_edges == 0:
            # a zero gradient, not None: a rank holding no edge of this relation still has to
            # reach the collective adjoints upstream (parallel.py's halo exchange)
            return g.new_zeros(ctx.csr.n_src, g.shape[1]), None
        return scatter_mean_bwd(g.contiguous(), ctx.csr), None


def mean_gather(x_src: torch.Tensor, csr: RelationCSR) -> torch.Tensor:
    """Differentiable K1 (forward) / K2 (backward) mean aggregation."""
    return _GatherMean.apply(x_src, csr)


# Gradients still being produced by an in-flight collective (parallel.py issues the adjoint of
# its post-table all-reduce asynchronously): the consumer below waits on the collective right
# before its first kernel, so the user-side backward kernels scheduled in between overlap it.
_PENDING: Dict[int, Tuple[torch.Tensor, object]] = {}


def defer_until(t: torch.Tensor, work) -> torch.Tensor:
    """Register ``t`` as not yet valid until ``work.wait()`` (a torch.distributed Work)."""
    _PENDING[id(t)] = (t, work)
    return t


def await_pending(t: torch.Tensor) -> torch.Tensor:
    entry = _PENDING.pop(id(t), None)
    if entry is not None and entry[0] is t:
        with torch.no_grad():
            entry[1].wait()   # NCCL: the current stream waits on the collective (no host sync)
    return t


def weighted_gather_raw(x_src: torch.Tensor, csr: RelationCSR, w_fwd: torch.Tensor,
                        row_w: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``out[i] = sum_{p in row i} w_fwd[p] x_src[col[p]]`` (K1 with per-edge weights).
    ``row_w``: the same weights when they are constant per row (w_fwd[p] = row_w[i], the
    sharded step's 1/deg_global): a source table of several GB is then gathered in
    source-block passes scaled per row (see :func:`gather_blocks`)."""
    x_src = _check_f32(x_src, "weighted_gather")
    out = torch.empty(csr.n_dst, x_src.shape[1], dtype=torch.float32, device=x_src.device)
    B = gather_blocks(x_src, csr.num_edges) if (row_w is not None and csr.num_edges) else 1
    if B > 1:
        passes, _ = csr.blocks("fwd", B)
        d, E = int(x_src.shape[1]), csr.num_edges
        _gather_blocked(x_src, passes, row_w, None, out, False,
                        f"gather_wfwd[{csr.n_dst}<-{csr.n_src}]x{d}",
                        gather_bytes(E, csr.n_dst, d, False),
                        gather_compulsory_bytes(E, csr.n_dst, csr.n_src, d, False))
        return out
    _gather(x_src, csr.fwd, None, csr_mean=False, out=out, accumulate=False, edge_w=w_fwd,
            kind="wfwd")
    return out


def weighted_scatter_bwd_raw(g: torch.Tensor, csr: RelationCSR, w_bwd: torch.Tensor,
                             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Transpose of :func:`weighted_gather_raw` over the CSC (K2), accumulating into ``out``."""
    acc = out is not None
    if out is None:
        out = torch.empty(csr.n_src, g.shape[1], dtype=torch.float32, device=g.device)
    _gather(g.contiguous(), csr.bwd, None, csr_mean=False, out=out, accumulate=acc, edge_w=w_bwd)
    return out


class _GatherWeighted(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_src, csr: RelationCSR, w_fwd, w_bwd):
        x_src = _check_f32(x_src, "weighted_gather")
        out = torch.empty(csr.n_dst, x_src.shape[1], dtype=torch.float32, device=x_src.device)
        _gather(x_src, csr.fwd, None, csr_mean=False, out=out, accumulate=False, edge_w=w_fwd,
                kind="wfwd")
        ctx.csr, ctx.w_bwd = csr, w_bwd
        return out

    @staticmethod
    def backward(ctx, g):
        await_pending(g)
        if not ctx.needs_input_grad[0]:
            return None, None, None, None
        csr = ctx.csr
        if csr.num_edges == 0:   # zero, not None: see _GatherMean.backward
            return g.new_zeros(csr.n_src, g.shape[1]), None, None, None
        out = torch.empty(csr.n_src, g.shape[1], dtype=torch.float32, device=g.device)
        _gather(g.contiguous(), csr.bwd, None, csr_mean=False, out=out, accumulate=False,
                edge_w=ctx.w_bwd)
        return out, None, None, None


def weighted_gather(x_src: torch.Tensor, csr: RelationCSR, w_fwd: torch.Tensor,
                    w_bwd: torch.Tensor) -> torch.Tensor:
    """``out[i] = sum_{p in row i} w_fwd[p] x_src[col[p]]`` (CSR order weights); backward walks
    the CSC with ``w_bwd`` (CSC order) — the same edge weights, transposed."""
    return _GatherWeighted.apply(x_src, csr, w_fwd, w_bwd)


class _FusedLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, relu: bool, w, b, *segs):
        segs = [_check_f32(s, "fused_linear") for s in segs]
        y = linear_fwd(segs, w.contiguous(), None if b is None else b.contiguous(), relu)
        ctx.relu, ctx.has_b = relu, b is not None
        ctx.save_for_backward(w, y, *segs)
        return y

    @staticmethod
    def backward(ctx, dy):
        await_pending(dy)    # a slice gradient whose reduce-scatter may be in flight (parallel.py)
        w, y, *segs = ctx.saved_tensors
        need = ctx.needs_input_grad
        dxs = [torch.empty_like(s) if need[3 + i] else None for i, s in enumerate(segs)]
        dw, db = linear_bwd(segs, w, dy.contiguous(), y if ctx.relu else None, dxs, need[1],
                            ctx.has_b and need[2])
        return (None, dw, db, *dxs)


def fused_linear(segs: Sequence[torch.Tensor], w: torch.Tensor, b: Optional[torch.Tensor],
                 relu: bool) -> torch.Tensor:
    """Differentiable K3: ``act(sum_s segs[s] @ w[:, seg s]^T + b)``."""
    return _FusedLinear.apply(relu, w, b, *segs)
