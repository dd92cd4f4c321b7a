"""GPU parity: every HIP kernel through the C ABI against the CPU oracle / golden fixtures.

Tolerances: integer CSR work bit-exact; fp32 paths within 1e-4 relative (north_star) — written as
``assert_close(rtol=1e-4, atol=1e-5 * scale)``.
"""
import contextlib
import pathlib

import numpy as np
import pytest
import torch

from oracle import csr_ref, sage_ref
from truth_recommendation_gnn_amd import (HeteroSAGE, SAGEConv, WeightedRGCN, WeightedRGCNAuthor,
                                          graph, ops, synth)

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = pathlib.Path(__file__).resolve().parent / "golden"
RTOL = 1e-4


def close(got, ref, rtol=RTOL, atol_scale=1e-5):
    got = got.detach().double().cpu()
    ref = torch.as_tensor(ref).detach().double().cpu()
    scale = max(float(ref.abs().max()) if ref.numel() else 0.0, 1e-6)
    torch.testing.assert_close(got, ref, rtol=rtol, atol=atol_scale * scale)


def rand_coo(rng, n_src, n_dst, E, skew=False):
    src = rng.integers(0, n_src, size=E)
    if skew:
        dst = synth._zipf_sample_np(rng, n_dst, E, 1.1)
    else:
        dst = rng.integers(0, n_dst, size=E)
    return torch.from_numpy(np.stack([src, dst]).astype(np.int64))


# ----------------------------------------------------------------------------- K5
@pytest.mark.parametrize("n_keys,E,skew", [(1, 10, False), (7, 0, False), (300, 5000, True),
                                           (70000, 200000, True), (1 << 17, 300000, False),
                                           (800000, 400000, True), (1000, 30000, True)])
def test_coo_to_csr_bit_exact(n_keys, E, skew):
    rng = np.random.default_rng(n_keys + E)
    ei = rand_coo(rng, 1000, n_keys, E, skew)
    g = graph.group_edges(ei[1].to(DEV), ei[0].to(DEV), n_keys, 1000)
    rowptr, col, perm = csr_ref.coo_to_csr(ei[1].numpy(), ei[0].numpy(), n_keys)
    assert np.array_equal(g.rowptr.cpu().numpy(), rowptr)
    assert np.array_equal(g.perm.cpu().numpy(), perm)
    assert np.array_equal(g.col.cpu().numpy(), col)


def test_coo_to_csr_rejects_out_of_range():
    ei = torch.tensor([[0, 5], [1, 2]], device=DEV)
    with pytest.raises(ValueError, match="out of range"):
        graph.group_edges(ei[1], ei[0], 3, 4)


def test_skew_plan_matches_reference_plan():
    rng = np.random.default_rng(3)
    ei = rand_coo(rng, 500, 50, 20000, skew=True)
    g = graph.group_edges(ei[1].to(DEV), ei[0].to(DEV), 50, 500, chunk=64)
    heavy, first = csr_ref.heavy_plan(g.rowptr.cpu().numpy(), 64)
    assert g.plan.n_heavy == heavy.size and g.plan.n_chunks == int(first[-1])
    assert np.array_equal(g.plan.heavy_rows.cpu().numpy(), heavy)
    assert np.array_equal(g.plan.heavy_first.cpu().numpy(), first)


# ----------------------------------------------------------------------------- K1 / K2
@pytest.mark.parametrize("d", [1, 3, 4, 7, 16, 64, 100, 128, 256, 300])
@pytest.mark.parametrize("chunk", [None, 8])
def test_gather_mean_matches_oracle(d, chunk):
    rng = np.random.default_rng(d)
    n_src, n_dst, E = 700, 300, 6000
    ei = rand_coo(rng, n_src, n_dst, E, skew=True)
    x = torch.from_numpy(rng.standard_normal((n_src, d)).astype(np.float32))
    ref = sage_ref.mean_aggregate(x, ei, n_dst)
    csr = graph.RelationCSR(ei.to(DEV), n_src, n_dst, chunk=chunk)
    got = ops.gather_mean(x.to(DEV), csr)
    close(got, ref)


@pytest.mark.parametrize("d", [3, 64, 128])
@pytest.mark.parametrize("chunk", [None, 16])
def test_scatter_mean_bwd_matches_autograd(d, chunk):
    rng = np.random.default_rng(10 + d)
    n_src, n_dst, E = 400, 900, 8000
    ei = rand_coo(rng, n_src, n_dst, E, skew=True)
    x = torch.from_numpy(rng.standard_normal((n_src, d)).astype(np.float32)).requires_grad_()
    g = torch.from_numpy(rng.standard_normal((n_dst, d)).astype(np.float32))
    sage_ref.mean_aggregate(x, ei, n_dst).backward(g)
    csr = graph.RelationCSR(ei.to(DEV), n_src, n_dst, chunk=chunk)
    got = ops.scatter_mean_bwd(g.to(DEV), csr)
    close(got, x.grad)
    acc = torch.ones(n_src, d, device=DEV)
    ops.scatter_mean_bwd(g.to(DEV), csr, out=acc)
    close(acc, x.grad + 1.0)


@pytest.mark.parametrize("d", [5, 64, 128])
@pytest.mark.parametrize("mode", [1, 2])
def test_score_gather_matches_float64(d, mode):
    """hgnn_score_gather: dP rows with each edge's weight recomputed from <U[u], P[row]>, heavy
    rows split into chunks (chunk=16 on a skewed graph)."""
    rng = np.random.default_rng(20 + d + mode)
    n_u, n_p, E = 600, 250, 9000
    ei = rand_coo(rng, n_u, n_p, E, skew=True)          # user -> post
    U = torch.from_numpy(rng.standard_normal((n_u, d)).astype(np.float32) * 0.3)
    P = torch.from_numpy(rng.standard_normal((n_p, d)).astype(np.float32) * 0.3)
    c, inv_e = 1.7, 1.0 / 12345
    s = (U.double()[ei[0]] * P.double()[ei[1]]).sum(1)
    sg = torch.sigmoid(s)
    w = c * inv_e * (sg - 1) if mode == 1 else inv_e * sg
    ref = torch.zeros(n_p, d, dtype=torch.float64).index_add_(0, ei[1], w[:, None] * U.double()[ei[0]])
    csr = graph.RelationCSR(ei.to(DEV), n_u, n_p, chunk=16)
    assert csr.fwd.plan.n_heavy > 0
    out = torch.full((n_p, d), 0.5, device=DEV)
    ops._score_gather(U.to(DEV), P.to(DEV), csr.fwd, mode, torch.tensor(c, device=DEV), inv_e,
                      out, True, "t")
    close(out, ref + 0.5)


@pytest.mark.parametrize("d", [5, 64, 128])
def test_score_gather2_matches_float64(d):
    """hgnn_score_gather2: positives (mode 1, heavy rows split with chunk=16) and negatives (mode 2)
    summed into one dP pass; includes posts with no positive or no negative edge."""
    rng = np.random.default_rng(40 + d)
    n_u, n_p, E = 600, 250, 9000
    pos = rand_coo(rng, n_u, n_p, E, skew=True)                  # Zipf head -> heavy rows
    neg = torch.stack([pos[0], torch.from_numpy(rng.integers(0, n_p - 10, E))])  # 10 posts unused
    U = torch.from_numpy(rng.standard_normal((n_u, d)).astype(np.float32) * 0.3)
    P = torch.from_numpy(rng.standard_normal((n_p, d)).astype(np.float32) * 0.3)
    c, inv_e = 1.7, 1.0 / 12345
    ref = torch.zeros(n_p, d, dtype=torch.float64)
    for ei, mode in ((pos, 1), (neg, 2)):
        sg = torch.sigmoid((U.double()[ei[0]] * P.double()[ei[1]]).sum(1))
        w = c * inv_e * (sg - 1) if mode == 1 else inv_e * sg
        ref.index_add_(0, ei[1], w[:, None] * U.double()[ei[0]])
    csr = graph.RelationCSR(pos.to(DEV), n_u, n_p, chunk=16)
    assert csr.fwd.plan.n_heavy > 0
    ncsr = graph.RelationCSR(neg.to(DEV), n_u, n_p, chunk=1 << 30)
    out = torch.full((n_p, d), 0.5, device=DEV)                 # every row must be written
    ops._score_gather2(U.to(DEV), P.to(DEV), csr.fwd, ncsr.fwd, torch.tensor(c, device=DEV),
                       inv_e, out)
    close(out, ref)


@pytest.mark.parametrize("d,slice_rows", [(64, 700), (128, 333), (4, 1200)])
def test_source_blocked_gathers_match_oracle(monkeypatch, d, slice_rows):
    """K1 mean and K2 as passes over source blocks (what gathers over multi-GB tables run, e.g.
    cfg4's 4.6 GB user table in 8 passes), forced here on small tables: each pass sums its block
    scaled by 1/deg of the whole relation into the output (skewed graph, heavy rows split per
    block, empty rows, accumulate mode) — against the oracle / autograd as the one-pass path."""
    monkeypatch.setattr(ops, "GATHER_BLOCK_BYTES", 1)
    monkeypatch.setattr(ops, "GATHER_BLOCK_SLICE", slice_rows * d * 4)
    rng = np.random.default_rng(77 + d)
    n_src, n_dst, E = 5000, 300, 60000
    ei = rand_coo(rng, n_src, n_dst, E, skew=True)
    ei = ei[:, ei[1] != 7]                                   # an empty destination row
    x = torch.from_numpy(rng.standard_normal((n_src, d)).astype(np.float32)).requires_grad_()
    csr = graph.RelationCSR(ei.to(DEV), n_src, n_dst, chunk=64)
    assert ops.gather_blocks(x) > 3
    ref = sage_ref.mean_aggregate(x, ei, n_dst)
    got = ops.gather_mean(x.detach().to(DEV), csr)
    close(got, ref)
    assert float(got[7].abs().max()) == 0.0
    passes, _ = csr.blocks("fwd", ops.gather_blocks(x))
    assert sum(p.plan.n_heavy for p in passes) > 0
    acc = torch.ones(n_dst, d, device=DEV)
    ops.gather_mean(x.detach().to(DEV), csr, out=acc)
    close(acc, ref + 1.0)
    # K2: blocks over the destinations' gradient rows (the table K2 reads)
    g = torch.from_numpy(rng.standard_normal((n_dst, d)).astype(np.float32))
    ref.backward(g)
    monkeypatch.setattr(ops, "GATHER_BLOCK_SLICE", 40 * d * 4)
    assert ops.gather_blocks(g) > 3
    close(ops.scatter_mean_bwd(g.to(DEV), csr), x.grad)
    acc = torch.full((n_src, d), 2.0, device=DEV)          # K2 accumulating into a buffer
    ops.scatter_mean_bwd(g.to(DEV), csr, out=acc)
    close(acc, x.grad + 2.0)


def test_gather_is_deterministic_bitwise():
    rng = np.random.default_rng(5)
    ei = rand_coo(rng, 5000, 200, 100000, skew=True).to(DEV)
    x = torch.randn(5000, 64, device=DEV)
    csr = graph.RelationCSR(ei, 5000, 200, chunk=64)
    a = ops.gather_mean(x, csr)
    b = ops.gather_mean(x, csr)
    assert torch.equal(a, b)


# ----------------------------------------------------------------------------- K3 / K4
@pytest.mark.parametrize("ks,h", [([64], 64), ([64, 64], 64), ([64, 64, 64], 64),
                                  ([128, 128], 128), ([3, 5], 7), ([16], 200), ([64, 4], 100),
                                  ([64], 128), ([32], 16), ([64, 32], 32), ([64, 64], 128),
                                  ([16, 48, 64], 64), ([32, 96], 64), ([48, 16], 128),
                                  ([128, 128], 64), ([64, 64, 128], 128), ([128], 128),
                                  ([128, 128, 128], 128), ([128, 128, 128, 128], 128),
                                  ([64, 256, 64], 128)])
@pytest.mark.parametrize("n", [1, 37, 1000, 20000])
def test_linear_fwd_bwd_matches_torch(ks, h, n):
    gen = torch.Generator().manual_seed(n + h)
    segs = [torch.randn(n, k, generator=gen) for k in ks]
    w = torch.randn(h, sum(ks), generator=gen) * 0.2
    b = torch.randn(h, generator=gen)
    dout = torch.randn(n, h, generator=gen)
    dsegs = [s.to(DEV) for s in segs]
    out = ops.linear_fwd(dsegs, w.to(DEV), b.to(DEV), relu=True)
    close(out, torch.relu(torch.cat(segs, 1) @ w.T + b))
    dxs = [torch.empty_like(s) for s in dsegs]
    dw, db = ops.linear_bwd(dsegs, w.to(DEV), dout.to(DEV), out, dxs, True, True)
    ref_dx, ref_dw, ref_db = _linear_bwd_ref(segs, w, dout, out)
    for gx, r in zip(dxs, ref_dx):
        close(gx, r)
    close(dw, ref_dw)
    close(db, ref_db)


def test_linear_general_kernels_at_many_row_blocks():
    """The general K3 kernels with 128-column tiles (>= 1024 workgroups: large N at shapes the
    compile-time kernels do not cover); smaller grids take 32-column tiles (the test above)."""
    n, ks, h = 140_000, [3, 5], 7
    gen = torch.Generator().manual_seed(5)
    segs = [torch.randn(n, k, generator=gen) for k in ks] + [torch.randn(n, 64, generator=gen)]
    w = torch.randn(200, 72, generator=gen) * 0.2
    b = torch.randn(200, generator=gen)
    dout = torch.randn(n, 200, generator=gen)
    dsegs = [s.to(DEV) for s in segs]
    out = ops.linear_fwd(dsegs, w.to(DEV), b.to(DEV), relu=True)
    close(out, torch.relu(torch.cat(segs, 1) @ w.T + b))
    dxs = [torch.empty_like(s) for s in dsegs]
    dw, db = ops.linear_bwd(dsegs, w.to(DEV), dout.to(DEV), out, dxs, True, True)
    ref_dx, ref_dw, ref_db = _linear_bwd_ref(segs, w, dout, out)
    for gx, r in zip(dxs, ref_dx):
        close(gx, r)
    close(dw, ref_dw)
    close(db, ref_db)


def _linear_bwd_ref(segs, w, dout, out_act):
    """float64 backward of relu(X W^T + b) given the kernel's forward output: the ReLU mask is
    taken from ``out_act`` itself, since a pre-activation within rounding of 0 may legitimately
    land on either side in fp32 and flip one row's dX by dout*W."""
    dz = dout.double()
    if out_act is not None:
        dz = dz * (out_act.detach().cpu() > 0)
    x = torch.cat(segs, 1).double()
    dx = dz @ w.double()
    return list(dx.split([s.shape[1] for s in segs], 1)), dz.T @ x, dz.sum(0)


@pytest.mark.parametrize("ks,h", [([64, 64], 64), ([64], 64), ([64, 64], 128), ([16, 48], 128),
                                  ([128, 128], 128), ([128, 128], 64), ([64, 64, 128], 128),
                                  ([128, 128, 128], 128), ([64, 256, 64], 128)])
@pytest.mark.parametrize("mode", ["no_relu", "dx_subset", "wgrad_only", "db_only", "dgrad_only"])
def test_linear_bwd_variants(ks, h, mode):
    """The compile-time-shape K3 backward (two-role, double-buffered tiles) under every operand
    combination the layers use: no activation mask, dX for a subset of segments, dW/db only."""
    n = 64 * 300 + 17
    gen = torch.Generator().manual_seed(7 * h + len(ks))
    segs = [torch.randn(n, k, generator=gen) for k in ks]
    w = torch.randn(h, sum(ks), generator=gen) * 0.2
    b = torch.randn(h, generator=gen)
    dout = torch.randn(n, h, generator=gen)
    relu = mode != "no_relu"
    z = torch.cat(segs, 1) @ w.T + b
    dsegs = [s.to(DEV) for s in segs]
    out = ops.linear_fwd(dsegs, w.to(DEV), b.to(DEV), relu=relu)
    close(out, torch.relu(z) if relu else z)
    ref_dx, ref_dw, ref_db = _linear_bwd_ref(segs, w, dout, out if relu else None)
    dxs = [torch.full_like(s, 7.0) for s in dsegs]
    if mode in ("wgrad_only", "db_only"):
        dxs = [None] * len(ks)
    elif mode == "dx_subset":
        dxs[0] = None
    need_w = mode not in ("db_only", "dgrad_only")
    need_b = mode != "dgrad_only"
    dw, db = ops.linear_bwd(dsegs, w.to(DEV), dout.to(DEV), out if relu else None, dxs,
                            need_w, need_b)
    for gx, r in zip(dxs, ref_dx):
        if gx is not None:
            close(gx, r)
    if need_w:
        close(dw, ref_dw)
    else:
        assert dw is None
    if need_b:
        close(db, ref_db)


@pytest.mark.parametrize("ks,h", [([64, 64], 64), ([64], 128), ([128, 128], 128), ([128], 128),
                                  ([16, 48], 128), ([3, 5], 7), ([64, 64, 128], 128),
                                  ([128, 128, 128], 128)])
@pytest.mark.parametrize("masked", [False, True])
def test_linear_bwd_dx_accumulate_bitwise(ks, h, masked):
    """hgnn_linear_bwd_ex's accumulate bits (dX added into what the buffer holds, for tables with
    two gradient producers — ops._pre_group_backward) give bitwise `held + dX` of the storing
    backward, in every kernel family (persistent dgrad v4/v5, the fused two-role backward, the
    general kernels), on the accumulated segments only."""
    n = 64 * 150 + 29
    gen = torch.Generator().manual_seed(11 * h + len(ks))
    dsegs = [torch.randn(n, k, generator=gen).to(DEV) for k in ks]
    w = (torch.randn(h, sum(ks), generator=gen) * 0.2).to(DEV)
    b = torch.randn(h, generator=gen).to(DEV)
    dout = torch.randn(n, h, generator=gen).to(DEV)
    mk = ops.relu_mask_for(n, h, masked, torch.device(DEV))
    out = ops.linear_fwd(dsegs, w, b, relu=masked, mask_out=mk)
    act = out if masked else None
    fresh = [torch.empty_like(x) for x in dsegs]
    dw0, db0 = ops.linear_bwd(dsegs, w, dout, act, fresh, True, True, mask=mk)
    held = [torch.randn(x.shape, generator=gen).to(DEV) for x in dsegs]
    acc = [t.clone() for t in held]
    add = [i % 2 == 0 for i in range(len(ks))]          # every other segment accumulates
    for i, a in enumerate(add):
        if not a:
            acc[i].fill_(123.0)                          # overwritten
    dw1, db1 = ops.linear_bwd(dsegs, w, dout, act, acc, True, True, mask=mk, dx_add=add)
    for i, a in enumerate(add):
        assert torch.equal(acc[i], held[i] + fresh[i] if a else fresh[i]), i
    assert torch.equal(dw0, dw1) and torch.equal(db0, db1)


def test_fuse_weights_multi_equals_per_update_calls():
    """hgnn_fuse_weights_multi / hgnn_split_weight_grads_multi (one launch each way for a
    layer's updates, round 6) against the per-update calls: three updates of different shapes
    (root + bias, no root, no bias, a shared parameter), outputs and every gradient bitwise."""
    gen = torch.Generator().manual_seed(11)
    h = 48
    p = lambda *shape: torch.randn(*shape, generator=gen).to(DEV).requires_grad_()  # noqa: E731
    shared = p(h, 64)
    groups = [([p(h, 64), p(h, 32)], [p(h, 64), shared], [p(h), p(h)], [1.0, 0.75]),
              ([p(h, 16)], [None], [p(h)], [0.5]),
              ([p(h, 64), shared, p(h, 8)], [p(h, 32), p(h, 32), None], [None, None, None],
               [1.75, 0.7, 0.3])]
    got = ops.fuse_weights_multi(groups)
    ref = [ops.fuse_weights(*g) for g in groups]
    params = list({id(t): t for g in groups for part in g[:3] for t in part
                   if t is not None}.values())
    loss, loss_ref = 0, 0
    for (W, b), (Wr, br) in zip(got, ref):
        assert torch.equal(W, Wr) and ((b is None and br is None) or torch.equal(b, br))
        gW = torch.randn(W.shape, generator=gen).to(DEV)
        loss = loss + (W * gW).sum()
        loss_ref = loss_ref + (Wr * gW).sum()
        if b is not None:
            gb = torch.randn(h, generator=gen).to(DEV)
            loss = loss + (b * gb).sum()
            loss_ref = loss_ref + (br * gb).sum()
    for a, r in zip(torch.autograd.grad(loss, params), torch.autograd.grad(loss_ref, params)):
        assert torch.equal(a, r)


@pytest.mark.parametrize("case", ["rgcn", "author", "no_root", "no_bias", "single"])
def test_fuse_weights_bitwise_equals_torch_expression(case):
    """hgnn_fuse_weights / hgnn_split_weight_grads against the torch expression they replace
    ([s_1 Wl_1 | ... | s_R Wl_R | sum_r s_r Wr_r], sum_r s_r bl_r): outputs and every parameter
    gradient bitwise equal."""
    gen = torch.Generator().manual_seed(len(case))
    scales = {"rgcn": [1.0, 0.75], "author": [1.75, 0.7, 0.3], "no_root": [1.0, 0.5],
              "no_bias": [0.75, 1.0], "single": [1.0]}[case]
    R, h = len(scales), 48
    ks = [64, 32, 64][:R]
    wl = [torch.randn(h, k, generator=gen).to(DEV).requires_grad_() for k in ks]
    wr = [None if (case == "no_root" and r == 1) else
          torch.randn(h, 64, generator=gen).to(DEV).requires_grad_() for r in range(R)]
    bl = [None if case == "no_bias" else torch.randn(h, generator=gen).to(DEV).requires_grad_()
          for _ in range(R)]
    W, b = ops.fuse_weights(wl, wr, bl, scales)
    # the torch expression (nn._fused_weights before round 2)
    w_ls, w_root, b_ref = [], None, None
    for r, s in enumerate(scales):
        sc = (lambda t: t) if s == 1.0 else (lambda t, s=s: t * s)
        w_ls.append(sc(wl[r]))
        if wr[r] is not None:
            w_root = sc(wr[r]) if w_root is None else w_root + sc(wr[r])
        if bl[r] is not None:
            b_ref = sc(bl[r]) if b_ref is None else b_ref + sc(bl[r])
    W_ref = torch.cat(w_ls + [w_root], 1)
    assert torch.equal(W, W_ref)
    assert (b is None and b_ref is None) or torch.equal(b, b_ref)
    params = [t for t in wl + wr + bl if t is not None]
    gW = torch.randn(W.shape, generator=gen).to(DEV)
    gb = torch.randn(h, generator=gen).to(DEV)
    loss = (W * gW).sum() + ((b * gb).sum() if b is not None else 0)
    got = torch.autograd.grad(loss, params)
    loss_ref = (W_ref * gW).sum() + ((b_ref * gb).sum() if b_ref is not None else 0)
    ref = torch.autograd.grad(loss_ref, params)
    for a, c in zip(got, ref):
        assert torch.equal(a, c)


def _unpack_relu_bits(mask, n, h):
    """The lane layout of hgnn_linear_fwd_mask as a dense [n, h] bool: word row*4 + g, bit 4c + e
    is column 16c + 4g + e."""
    m = mask.cpu().view(torch.int32).numpy().astype(np.uint32).reshape(n, 4)
    out = np.zeros((n, h), dtype=bool)
    for g in range(4):
        for c in range(h // 16):
            for e in range(4):
                out[:, 16 * c + 4 * g + e] = (m[:, g] >> np.uint32(4 * c + e)) & 1
    return out


@pytest.mark.parametrize("ks,h", [([128, 128], 128), ([128], 128), ([64, 64], 64),
                                  ([64, 64, 128], 128), ([16, 48], 128), ([64], 48),
                                  ([64, 64], 112), ([128, 128, 128], 128)])
@pytest.mark.parametrize("mode", ["all", "wgrad_only", "dz_out"])
def test_linear_relu_bits_equal_float_mask(ks, h, mode):
    """hgnn_linear_fwd_mask writes out > 0 as bits (persistent kernels, or k_relu_mask for other
    shapes: h = 48, 112) and hgnn_linear_bwd_mask with those bits gives bitwise the gradients of
    the float-mask backward (hgnn_linear_bwd_dz), dz side output included."""
    n = 64 * 300 + 17
    gen = torch.Generator().manual_seed(3 * h + len(ks))
    segs = [torch.randn(n, k, generator=gen).to(DEV) for k in ks]
    w = (torch.randn(h, sum(ks), generator=gen) * 0.2).to(DEV)
    b = torch.randn(h, generator=gen).to(DEV)
    dout = torch.randn(n, h, generator=gen).to(DEV)
    mk = ops.relu_mask_for(n, h, True, torch.device(DEV))
    assert mk is not None
    out = ops.linear_fwd(segs, w, b, relu=True, mask_out=mk)
    ref = ops.linear_fwd(segs, w, b, relu=True)
    assert torch.equal(out, ref)
    np.testing.assert_array_equal(_unpack_relu_bits(mk, n, h), (out > 0).cpu().numpy())
    res = []
    for m in (None, mk):
        dxs = [None] * len(ks) if mode == "wgrad_only" else [torch.empty_like(x) for x in segs]
        dz = torch.empty_like(dout) if mode == "dz_out" else None
        dw, db = ops.linear_bwd(segs, w, dout, out, dxs, True, True, dz_out=dz, mask=m)
        res.append([dw, db, dz] + dxs)
    for a, c in zip(*res):
        if a is not None:
            assert torch.equal(a, c)


# ----------------------------------------------------------------------------- models
def _fixture_cfg1():
    z = np.load(GOLD / "cfg1_weighted_rgcn.npz")
    x = {"user": torch.from_numpy(z["x_user"]).to(DEV), "post": torch.from_numpy(z["x_post"]).to(DEV)}
    e = {synth.SOCIAL: torch.from_numpy(z["ei_social"]).to(DEV),
         synth.ENGAGES: torch.from_numpy(z["ei_engages"]).to(DEV),
         synth.REV_ENGAGES: torch.from_numpy(z["ei_rev_engages"]).to(DEV)}
    params = {k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param:")}
    return z, x, e, params


def test_weighted_rgcn_train_step_matches_golden():
    z, x, e, params = _fixture_cfg1()
    model = WeightedRGCN(hidden_dim=64).to(DEV)
    model.load_state_dict(params)
    out = model(x, e)
    close(out["user"], z["out_user"])
    close(out["post"], z["out_post"])
    pos = e[synth.ENGAGES]
    loss = ops.link_loss(out["user"], out["post"], pos, torch.from_numpy(z["neg_p"]).to(DEV),
                         torch.from_numpy(z["pos_weights"]).to(DEV))
    assert abs(float(loss.detach()) - float(z["loss"])) <= RTOL * abs(float(z["loss"]))
    loss.backward()
    for name, p in model.named_parameters():
        close(p.grad, z["grad:" + name])


def test_hetero_sage_two_layer_matches_golden():
    z = np.load(GOLD / "cfg2_slice_hetero_sage.npz")
    ei = torch.from_numpy(z["ei_engages"]).to(DEV)
    e = {synth.ENGAGES: ei, synth.REV_ENGAGES: ei.flip(0)}
    x = {"user": torch.from_numpy(z["x_user"]).to(DEV), "post": torch.from_numpy(z["x_post"]).to(DEV)}
    rels = [(synth.REV_ENGAGES, 1.0), (synth.ENGAGES, 1.0)]
    model = HeteroSAGE(64, rels, num_layers=2).to(DEV)
    params = {k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param:")}
    model.load_state_dict(params)
    out = model(x, e)
    close(out["user"], z["out_user"])
    close(out["post"], z["out_post"])
    loss = ops.link_loss(out["user"], out["post"], ei, torch.from_numpy(z["neg_p"]).to(DEV),
                         torch.from_numpy(z["pos_weights"]).to(DEV))
    assert abs(float(loss.detach()) - float(z["loss"])) <= RTOL * abs(float(z["loss"]))
    loss.backward()
    for name, p in model.named_parameters():
        close(p.grad, z["grad:" + name])


@pytest.mark.parametrize("fixture,d", [("cfg2_slice_hetero_sage.npz", 64),
                                       ("cfg3_slice_hetero_sage.npz", 128)])
def test_hetero_sage_two_layer_fused_loss_matches_golden(fixture, d):
    """The training step as bench.py runs it — 2-layer model, the fused link loss (scoring pass,
    negatives sort, score-recomputing dP gather) driving the backward — at d = h = 64 and at the
    BASELINE cfg3/cfg4 width d = h = 128 (K=256 projection variants, d=128 gathers)."""
    z = np.load(GOLD / fixture)
    ei = torch.from_numpy(z["ei_engages"]).to(DEV)
    e = {synth.ENGAGES: ei, synth.REV_ENGAGES: ei.flip(0)}
    x = {"user": torch.from_numpy(z["x_user"]).to(DEV), "post": torch.from_numpy(z["x_post"]).to(DEV)}
    assert x["user"].shape[1] == d
    rels = [(synth.REV_ENGAGES, 1.0), (synth.ENGAGES, 1.0)]
    model = HeteroSAGE(d, rels, num_layers=2).to(DEV)
    model.load_state_dict({k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param:")})
    out = model(x, e)
    close(out["user"], z["out_user"])
    close(out["post"], z["out_post"])
    loss = ops.edge_bce_loss(out["user"], out["post"], ei, torch.from_numpy(z["neg_p"]).to(DEV),
                             torch.from_numpy(z["pos_weights"]).to(DEV))
    assert abs(float(loss.detach()) - float(z["loss"])) <= RTOL * abs(float(z["loss"]))
    loss.backward()
    for name, p in model.named_parameters():
        close(p.grad, z["grad:" + name])


def test_fused_loss_second_backward_through_retained_graph():
    """A retained graph back-propagated twice gives the same gradients both times (the second
    backward recomputes dU/dP; the first handed its buffers on, scaled in place), as the torch
    loss does: the leaves accumulate g1 + g2."""
    z = np.load(GOLD / "cfg2_slice_hetero_sage.npz")
    ei = torch.from_numpy(z["ei_engages"]).to(DEV)
    U = torch.from_numpy(z["out_user"]).to(DEV).requires_grad_()
    P = torch.from_numpy(z["out_post"]).to(DEV).requires_grad_()
    loss = ops.edge_bce_loss(U, P, ei, torch.from_numpy(z["neg_p"]).to(DEV),
                             torch.from_numpy(z["pos_weights"]).to(DEV))
    (2.0 * loss).backward(retain_graph=True)
    g1u, g1p = U.grad.clone(), P.grad.clone()
    loss.backward(retain_graph=True)
    g2u, g2p = U.grad - g1u, P.grad - g1p
    loss.backward()
    U2 = U.detach().clone().requires_grad_()
    P2 = P.detach().clone().requires_grad_()
    ref = ops.link_loss(U2, P2, ei, torch.from_numpy(z["neg_p"]).to(DEV),
                        torch.from_numpy(z["pos_weights"]).to(DEV))
    (2.0 * ref).backward()
    close(g1u, U2.grad)
    close(g1p, P2.grad)
    close(g2u, 0.5 * U2.grad)
    close(g2p, 0.5 * P2.grad)
    close(U.grad, 2.0 * U2.grad)     # 2 + 1 + 1


def test_sage_conv_standalone_and_homogeneous_input():
    rng = np.random.default_rng(1)
    ei = rand_coo(rng, 50, 50, 400)
    x = torch.from_numpy(rng.standard_normal((50, 12)).astype(np.float32))
    conv = SAGEConv(12, 9).to(DEV)
    xg = x.to(DEV).requires_grad_()
    out = conv(xg, ei.to(DEV))
    W = {k: v.detach().cpu() for k, v in conv.state_dict().items()}
    xr = x.clone().requires_grad_()
    ref = sage_ref.sage_conv(xr, xr, ei, W["lin_l.weight"], W["lin_l.bias"], W["lin_r.weight"])
    close(out, ref)
    g = torch.randn(50, 9)
    out.backward(g.to(DEV))
    ref.backward(g)
    close(xg.grad, xr.grad)


def test_inductive_single_user_zero_edges():
    # inference.py:410-424: one user, post table [0, 64], every relation E=0
    z, _, _, params = _fixture_cfg1()
    model = WeightedRGCN(64).to(DEV)
    model.load_state_dict(params)
    empty = torch.empty(2, 0, dtype=torch.long, device=DEV)
    xu = torch.randn(1, 64, device=DEV)
    e = {synth.SOCIAL: empty, synth.ENGAGES: empty.clone(), synth.REV_ENGAGES: empty.clone()}
    with torch.no_grad():
        out = model({"user": xu, "post": torch.empty(0, 64, device=DEV)}, e)
    P = {k: v for k, v in params.items()}
    ref_u = torch.relu(1.0 * (P["msg_direct.lin_l.bias"] + xu.cpu() @ P["msg_direct.lin_r.weight"].T)
                       + 0.75 * (P["msg_social.lin_l.bias"] + xu.cpu() @ P["msg_social.lin_r.weight"].T))
    close(out["user"], ref_u)
    assert out["post"].shape == (0, 64)


def test_author_variant_matches_oracle():
    g = synth.make_graph("cfg1")
    e = dict(g.edge_index_dict)
    e[("post", "followed_by", "user")] = torch.empty(2, 0, dtype=torch.long)  # test_gnn.py:103-106
    model = WeightedRGCNAuthor(64).to(DEV)
    x = {k: v.to(DEV) for k, v in g.x_dict.items()}
    out = model(x, {k: v.to(DEV) for k, v in e.items()})
    params = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    ref = sage_ref.weighted_rgcn(params, g.x_dict, e, layout=sage_ref.TEST_LAYOUT)
    close(out["user"], ref["user"])
    close(out["post"], ref["post"])


# ----------------------------------------------------------------------------- full-size properties
def test_cfg2_full_size_linearity_checksum():
    """At BASELINE config 2 size (20M edges): sum_i deg_i * aggr_i == sum_e x_src[src_e]
    (a checksum of checksums, float64), and the CSR row lengths equal the COO degree counts."""
    g = synth.make_graph("cfg2", device=DEV)
    ei = g.edge_index_dict[synth.ENGAGES]
    csr = graph.RelationCSR(ei, g.num_users, g.num_posts)
    deg = torch.bincount(ei[1], minlength=g.num_posts)
    assert torch.equal((csr.fwd.rowptr[1:] - csr.fwd.rowptr[:-1]).long(), deg)
    agg = ops.gather_mean(g.x_dict["user"], csr)
    lhs = (agg.double() * deg.double()[:, None]).sum(0)
    outdeg = torch.bincount(ei[0], minlength=g.num_users).double()
    rhs = (g.x_dict["user"].double() * outdeg[:, None]).sum(0)
    torch.testing.assert_close(lhs, rhs, rtol=1e-6, atol=1e-3)
    assert csr.fwd.plan.n_heavy > 0   # the Zipf head really exercised the chunked path


# ----------------------------------------------------------------------------- fused link loss
@pytest.mark.parametrize("d", [64, 128, 5, 200, 16])
def test_edge_bce_loss_matches_oracle(d):
    rng = np.random.default_rng(100 + d)
    nu, npost, E = 300, 120, 5000
    pos = torch.from_numpy(np.stack([rng.integers(0, nu, E),
                                     synth._zipf_sample_np(rng, npost, E, 0.9)]).astype(np.int64))
    neg = torch.from_numpy(rng.integers(0, npost, E).astype(np.int64))
    pw = torch.from_numpy(np.where(rng.random(E) < 0.3, 3.0, 1.0).astype(np.float32))
    U = torch.from_numpy(rng.standard_normal((nu, d)).astype(np.float32) * 0.3)
    P = torch.from_numpy(rng.standard_normal((npost, d)).astype(np.float32) * 0.3)
    Ur, Pr = U.clone().requires_grad_(), P.clone().requires_grad_()
    ref = sage_ref.link_loss(Ur, Pr, pos, neg, pw)
    (ref * 2.5).backward()
    Ud, Pd = U.to(DEV).requires_grad_(), P.to(DEV).requires_grad_()
    pos_d = pos.to(DEV)
    got = ops.edge_bce_loss(Ud, Pd, pos_d, neg.to(DEV), pw.to(DEV))
    (got * 2.5).backward()
    close(got, ref)
    close(Ud.grad, Ur.grad)
    close(Pd.grad, Pr.grad)
    # same draws presented in the user-grouped order give the same loss
    csr = graph.relation_csr(pos_d, nu, npost)
    neg_u = ops.negatives_in_user_order(csr, neg.to(DEV))
    got2 = ops.edge_bce_loss(Ud.detach(), Pd.detach(), pos_d, neg_u, pw.to(DEV), neg_order="user")
    assert torch.equal(got2, got.detach())


def test_edge_bce_loss_rejects_bad_negatives():
    pos = torch.tensor([[0, 1], [0, 1]], device=DEV)
    U, P = torch.randn(2, 8, device=DEV), torch.randn(2, 8, device=DEV)
    with pytest.raises(ValueError, match="out of range"):
        ops.edge_bce_loss(U, P, pos, torch.tensor([0, 7], device=DEV), torch.ones(2, device=DEV))
    with pytest.raises(ValueError, match="out of range"):       # int32 path: no pre-sort check
        ops.edge_bce_loss(U, P, pos, torch.tensor([7, 0], dtype=torch.int32, device=DEV),
                          torch.ones(2, device=DEV))


@pytest.mark.parametrize("d", [64, 16])
def test_edge_bce_loss_int32_negatives_bitwise_equal(d):
    """int32 negatives (sample_negatives) take the validation-free sort and the int32 scoring
    entry; the same draws as int64 give bitwise the same loss and gradients."""
    rng = np.random.default_rng(7 + d)
    nu, npost, E = 400, 150, 8000
    pos = torch.from_numpy(np.stack([rng.integers(0, nu, E),
                                     synth._zipf_sample_np(rng, npost, E, 0.9)]).astype(np.int64))
    neg = torch.from_numpy(rng.integers(0, npost, E).astype(np.int64)).to(DEV)
    pw = torch.ones(E, device=DEV)
    U = torch.from_numpy(rng.standard_normal((nu, d)).astype(np.float32)).to(DEV)
    P = torch.from_numpy(rng.standard_normal((npost, d)).astype(np.float32)).to(DEV)
    res = []
    for n in (neg, neg.to(torch.int32)):
        Ud, Pd = U.clone().requires_grad_(), P.clone().requires_grad_()
        loss = ops.edge_bce_loss(Ud, Pd, pos.to(DEV), n, pw)
        loss.backward()
        res.append((loss.detach(), Ud.grad, Pd.grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_sample_negatives_uniform_and_seeded():
    pos = torch.zeros(2, 400_000, dtype=torch.int64, device=DEV)
    g1 = torch.Generator(device=DEV).manual_seed(3)
    a = ops.sample_negatives(pos, 1000, generator=g1)
    b = ops.sample_negatives(pos, 1000, generator=torch.Generator(device=DEV).manual_seed(3))
    c = ops.sample_negatives(pos, 1000, generator=g1)              # the generator advanced
    assert a.dtype == torch.int32 and torch.equal(a, b) and not torch.equal(a, c)
    assert int(a.min()) >= 0 and int(a.max()) < 1000
    counts = torch.bincount(a.long(), minlength=1000).double()
    chi2 = float(((counts - 400.0) ** 2 / 400.0).sum())             # 999 dof: mean 999, sd ~45
    assert 800 < chi2 < 1200
    lag = (a[1:].double() - 499.5) * (a[:-1].double() - 499.5)      # no serial correlation
    assert abs(float(lag.mean())) / (1000 ** 2 / 12) < 0.01


@pytest.mark.parametrize("E,n_keys", [(0, 7), (1, 1), (1000, 1), (5000, 37),
                                      (300_000, 100_000), (2_000_000, 1_000_000),
                                      (1_000_003, 2**21 + 5),     # > 2^20 keys: LSD sort
                                      (3_000_000, 2**20), (3 * 16384 + 5, 2**20 + 1),
                                      (16384 * 5, 1000), (12_345, 2**17),
                                      (70_000_001, 1_000_000)])   # > 2^26 draws, ragged last tile
def test_draw_sort_negatives_is_draw_then_sort(E, n_keys):
    """hgnn_draw_sort_negatives (draws computed inside the sort's first pass) is bit for bit
    hgnn_uniform_i32 followed by hgnn_sort_pairs_i32 (the LSD radix sort), and a stable sort
    (numpy) of the draws."""
    from truth_recommendation_gnn_amd import _native as Nn
    lib, s = Nn.lib(), Nn.stream_ptr(torch.device(DEV))
    seed = torch.tensor([0x1234_5678_9ABC_DEF], dtype=torch.int64, device=DEV)
    uop = torch.sort(torch.randint(0, 1 << 24, (E,), device=DEV, dtype=torch.int32))[0]
    ws = Nn.workspace(lib.hgnn_sort_pairs_ws_bytes(E, n_keys), torch.device(DEV))
    neg = torch.full((E,), -1, dtype=torch.int32, device=DEV)
    rp = torch.empty(n_keys + 1, dtype=torch.int32, device=DEV)
    us = torch.empty(E, dtype=torch.int32, device=DEV)
    Nn.check(lib.hgnn_draw_sort_negatives(Nn.ptr(seed), Nn.ptr(uop), E, n_keys, Nn.ptr(neg),
                                          Nn.ptr(rp), Nn.ptr(us), Nn.ptr(ws), ws.numel(), s),
             "hgnn_draw_sort_negatives")
    neg2 = torch.empty(E, dtype=torch.int32, device=DEV)
    rp2 = torch.empty(n_keys + 1, dtype=torch.int32, device=DEV)
    us2 = torch.empty(E, dtype=torch.int32, device=DEV)
    if E:
        Nn.check(lib.hgnn_uniform_i32(Nn.ptr(seed), E, n_keys, Nn.ptr(neg2), s), "uniform")
    Nn.check(lib.hgnn_sort_pairs_i32(Nn.ptr(neg2), Nn.ptr(uop), None, E, n_keys, Nn.ptr(rp2),
                                     Nn.ptr(us2), None, None, Nn.ptr(ws), ws.numel(), s), "sort")
    torch.cuda.synchronize()
    assert torch.equal(neg, neg2) and torch.equal(rp, rp2) and torch.equal(us, us2)
    k = neg.cpu().numpy().astype(np.int64)
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(us.cpu().numpy(), uop.cpu().numpy()[order])
    np.testing.assert_array_equal(rp.cpu().numpy(),
                                  np.searchsorted(k[order], np.arange(n_keys + 1), side="left"))


def test_fused_loss_negative_draw_equals_materialised():
    """edge_bce_loss with a NegativeDraw (draw + grouping in one call) gives bitwise the loss and
    gradients of the same draws materialised first (NegativeDraw.tensor())."""
    z, x, e, params = _fixture_cfg1()
    model = WeightedRGCN(hidden_dim=64).to(DEV)
    model.load_state_dict(params)
    with torch.no_grad():
        out = model(x, e)
    pos = e[synth.ENGAGES]
    pw = torch.from_numpy(z["pos_weights"]).to(DEV)
    dr = ops.draw_negatives(pos, out["post"].shape[0],
                            generator=torch.Generator(device=DEV).manual_seed(11))
    csr = ops.relation_csr_for_loss(pos, out["user"].shape[0], out["post"].shape[0])
    res = []
    for n in (dr, dr.tensor()):
        U, P = out["user"].clone().requires_grad_(), out["post"].clone().requires_grad_()
        loss = ops.edge_bce_loss(U, P, pos, n, pw, neg_order="user")
        loss.backward()
        res.append((loss.detach(), U.grad, P.grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    # and the torch reference on the same draws, put back in COO edge order
    neg_user = dr.tensor().long()
    neg_edge = torch.empty_like(neg_user)
    neg_edge[csr.bwd.perm.long()] = neg_user
    U, P = out["user"].clone().requires_grad_(), out["post"].clone().requires_grad_()
    ref = ops.link_loss(U, P, pos, neg_edge, pw)
    ref.backward()
    close(res[0][0], ref.detach())
    close(res[0][1], U.grad)
    close(res[0][2], P.grad)
    with pytest.raises(ValueError):
        ops.edge_bce_loss(out["user"], out["post"], pos, dr, pw, neg_order="edge")


@pytest.mark.parametrize("neg_kind", ["int32", "draw"])
def test_autograd_loss_presorted_on_side_stream_is_bitwise(neg_kind):
    """edge_bce_loss(presorted=...) with the grouping done ahead on a side stream (the bench's N = 1
    step) gives bitwise the loss and gradients of the grouping inside the loss; presorted
    negatives of other draws are refused."""
    z, x, e, params = _fixture_cfg1()
    model = WeightedRGCN(hidden_dim=64).to(DEV)
    model.load_state_dict(params)
    with torch.no_grad():
        out = model(x, e)
    pos = e[synth.ENGAGES]
    pw = torch.from_numpy(z["pos_weights"]).to(DEV)
    nu, np_ = out["user"].shape[0], out["post"].shape[0]
    dr = ops.draw_negatives(pos, np_, generator=torch.Generator(device=DEV).manual_seed(5))
    neg = dr if neg_kind == "draw" else dr.tensor()
    res = []
    for presort in (False, True):
        U, P = out["user"].clone().requires_grad_(), out["post"].clone().requires_grad_()
        pre = None
        if presort:
            main, side = torch.cuda.current_stream(DEV), torch.cuda.Stream(DEV)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                pre = ops.presort_negatives(nu, np_, pos, neg, "user")
            pre.rowptr.record_stream(main)
            pre.users.record_stream(main)
            main.wait_stream(side)
        loss = ops.edge_bce_loss(U, P, pos, neg, pw, neg_order="user", presorted=pre)
        loss.backward()
        res.append((loss.detach(), U.grad, P.grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    other = ops.draw_negatives(pos, np_, generator=torch.Generator(device=DEV).manual_seed(6))
    with pytest.raises(ValueError, match="other draws"):
        ops.edge_bce_loss(out["user"], out["post"], pos, other, pw, neg_order="user",
                          presorted=pre)
    if neg_kind == "int32":
        # the same draws read in the other order: the error names both orders
        with pytest.raises(ValueError, match="neg_order='user'.*neg_order='edge'"):
            ops.edge_bce_loss(out["user"], out["post"], pos, neg, pw, neg_order="edge",
                              presorted=pre)


@pytest.mark.parametrize("neg_kind", ["int32", "draw"])
def test_loss_dp_gather_in_row_blocks_is_bitwise_one_pass(neg_kind):
    """The sharded step's dP gather over the post table as it lands in row blocks (p_chunks: each
    block's positives a rowptr slice with its own skew plan, _row_range) gives bitwise the loss,
    dU and dP of the one-pass gather — blocks in any order, an empty block, heavy (chunked) rows
    inside blocks and on their edges; int32 negatives and the in-kernel NegativeDraw."""
    rng = np.random.default_rng(21)
    nu, npost, E, d = 5000, 3000, 400_000, 64
    pos = torch.from_numpy(np.stack([rng.integers(0, nu, E),
                                     synth._zipf_sample_np(rng, npost, E, 1.0)]).astype(np.int64)
                           ).to(DEV)
    U = torch.from_numpy(rng.standard_normal((nu, d)).astype(np.float32) * 0.3).to(DEV)
    P = torch.from_numpy(rng.standard_normal((npost, d)).astype(np.float32) * 0.3).to(DEV)
    cscale = torch.tensor(1.25, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(4)
    neg = (ops.sample_negatives(pos, npost, generator=gen) if neg_kind == "int32"
           else ops.draw_negatives(pos, npost, generator=gen))
    csr = ops.relation_csr_for_loss(pos, nu, npost)
    heavy = sorted(set(csr.fwd.plan.heavy_rows.cpu().tolist()))
    assert len(heavy) >= 3                      # the Zipf head really is chunked
    h0 = heavy[len(heavy) // 2]
    a, b = h0, max(h0 + 1, (h0 + npost) // 2)   # a block starting on a heavy row
    ref = ops.edge_bce_loss_raw(U, P, pos, neg, E, cscale)
    for chunks in ([(a, b, None), (0, a, None), (b, b, None), (b, npost, None)],
                   [(0, npost, None)],
                   [(q * npost // 7, (q + 1) * npost // 7, None) for q in range(7)]):
        got = ops.edge_bce_loss_raw(U, P, pos, neg, E, cscale, p_chunks=chunks)
        for x, y in zip(got, ref):
            assert torch.equal(x, y)


@pytest.mark.parametrize("nu,npost,E,d", [(3000, 1 << 20, 70_001, 128), (500, 37, 9_000, 64),
                                           (10, 5, 0, 16)])
def test_edge_score_draw_entry_equals_materialised_draws(nu, npost, E, d):
    """hgnn_edge_score_fwd_draw (each position's negative drawn in the kernel) is bit for bit
    hgnn_edge_score_fwd_i32 over the draws hgnn_uniform_i32 materialises from the same seed."""
    from truth_recommendation_gnn_amd import _native as Nn
    lib, s = Nn.lib(), Nn.stream_ptr(torch.device(DEV))
    g = torch.Generator(device=DEV).manual_seed(5)
    users = torch.sort(torch.randint(0, nu, (E,), device=DEV, generator=g))[0]
    rowptr = torch.searchsorted(users, torch.arange(nu + 1, device=DEV)).to(torch.int32)
    col = torch.randint(0, npost, (E,), device=DEV, generator=g, dtype=torch.int32)
    U = torch.randn(nu, d, device=DEV, generator=g)
    P = torch.randn(npost, d, device=DEV, generator=g)
    c = torch.tensor(1.25, device=DEV)
    seed = torch.tensor([0x0BAD_5EED_1234], dtype=torch.int64, device=DEV)
    neg = torch.empty(E, dtype=torch.int32, device=DEV)
    if E:
        Nn.check(lib.hgnn_uniform_i32(Nn.ptr(seed), E, npost, Nn.ptr(neg), s), "uniform")
    outs = []
    for entry in ("draw", "i32"):
        dU = torch.full_like(U, float("nan"))
        part = torch.empty(int(lib.hgnn_edge_score_parts(nu)), device=DEV)
        loss = torch.empty((), device=DEV)
        err = torch.zeros(2, dtype=torch.int32, device=DEV)
        if entry == "draw":
            rc = lib.hgnn_edge_score_fwd_draw(Nn.ptr(U), Nn.ptr(P), d, nu, npost, Nn.ptr(rowptr),
                                              Nn.ptr(col), Nn.ptr(seed), E, Nn.ptr(c), Nn.ptr(dU),
                                              Nn.ptr(part), Nn.ptr(loss), Nn.ptr(err), s)
        else:
            rc = lib.hgnn_edge_score_fwd_i32(Nn.ptr(U), Nn.ptr(P), d, nu, npost, Nn.ptr(rowptr),
                                             Nn.ptr(col), Nn.ptr(neg) if E else None, E,
                                             Nn.ptr(c), Nn.ptr(dU), Nn.ptr(part), Nn.ptr(loss),
                                             Nn.ptr(err), s)
        Nn.check(rc, entry)
        torch.cuda.synchronize()
        assert int(err[0]) == 0
        outs.append((loss, dU))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    if E:
        assert lib.hgnn_edge_score_fwd_draw(Nn.ptr(U), Nn.ptr(P), d, nu, npost, Nn.ptr(rowptr),
                                            Nn.ptr(col), None, E, Nn.ptr(c), Nn.ptr(dU),
                                            Nn.ptr(part), Nn.ptr(loss), Nn.ptr(err), s) != 0


def test_weighted_rgcn_fused_loss_step_matches_golden():
    z, x, e, params = _fixture_cfg1()
    model = WeightedRGCN(hidden_dim=64).to(DEV)
    model.load_state_dict(params)
    out = model(x, e)
    loss = ops.edge_bce_loss(out["user"], out["post"], e[synth.ENGAGES],
                             torch.from_numpy(z["neg_p"]).to(DEV),
                             torch.from_numpy(z["pos_weights"]).to(DEV))
    assert abs(float(loss.detach()) - float(z["loss"])) <= RTOL * abs(float(z["loss"]))
    loss.backward()
    for name, p in model.named_parameters():
        close(p.grad, z["grad:" + name])


# digit plans (csr_build.hip radix_plan): under 2^20 pairs the fewest passes of up to 10 bits,
# one-tile sorts (<= 8192 pairs) without count / scan kernels; larger sorts by the cost table
@pytest.mark.parametrize("E,nk", [(100000, 70000),       # 17 bits: 2 passes of 9
                                  (300000, 800000),      # 20 bits: 2 passes of 10
                                  (200000, 300000),      # 19 bits: 2 passes of 10 (last 9)
                                  (5000, 900),           # 10 bits: 1 pass, one tile
                                  (50000, 3_000_000),    # 22 bits: 3 passes of 8
                                  (8192, 1000),          # exactly one tile
                                  (8000, 2**20 - 1),     # one tile, 20 bits: 2 passes of 10
                                  (1, 5), (64, 3),       # one tile, a few items
                                  (8193, 100),           # one item in a second tile
                                  (2_500_001, 100_000),  # 17 bits by the cost table, ragged tail
                                  (2**26 + 3, 1_000_000),  # > 2^26 keys, two payloads
                                  (40000, -1)])          # every key equal: one digit holds all
def test_sort_pairs_matches_numpy(E, nk):
    rng = np.random.default_rng(9 + abs(nk))
    if nk < 0:
        nk = 5000
        keys = torch.full((E,), 4321, dtype=torch.int32)
    else:
        keys = torch.from_numpy(rng.integers(0, nk, E).astype(np.int32))
    a = torch.arange(E, dtype=torch.int32)
    b = torch.from_numpy(rng.integers(-5, 5, E).astype(np.int32))
    from truth_recommendation_gnn_amd import _native as Nn
    dev = torch.device(DEV)
    rowptr = torch.empty(nk + 1, dtype=torch.int32, device=dev)
    ao = torch.empty(E, dtype=torch.int32, device=dev)
    bo = torch.empty(E, dtype=torch.int32, device=dev)
    inv = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = Nn.workspace(Nn.lib().hgnn_sort_pairs_ws_bytes(E, nk), dev)
    kd, ad, bd = keys.to(dev), a.to(dev), b.to(dev)
    Nn.check(Nn.lib().hgnn_sort_pairs_i32(Nn.ptr(kd), Nn.ptr(ad), Nn.ptr(bd), E, nk, Nn.ptr(rowptr),
                                          Nn.ptr(ao), Nn.ptr(bo), Nn.ptr(inv), Nn.ptr(ws), ws.numel(),
                                          Nn.stream_ptr(dev)), "sort")
    order = np.argsort(keys.numpy(), kind="stable")
    assert np.array_equal(ao.cpu().numpy(), order)
    assert np.array_equal(bo.cpu().numpy(), b.numpy()[order])
    rp, _, _ = csr_ref.coo_to_csr(keys.numpy(), keys.numpy(), nk)
    assert np.array_equal(rowptr.cpu().numpy(), rp)


# ----------------------------------------------------------------------------- sharded path
def test_user_shard_world1_matches_fused_model_and_oracle():
    """parallel.UserShard on the HIP kernels (world=1, identity collectives) reproduces the fused
    single-GPU model and the oracle: outputs, loss, gradients."""
    from truth_recommendation_gnn_amd import parallel
    z = np.load(GOLD / "cfg2_slice_hetero_sage.npz")
    ei = torch.from_numpy(z["ei_engages"]).to(DEV)
    x = {"user": torch.from_numpy(z["x_user"]).to(DEV), "post": torch.from_numpy(z["x_post"]).to(DEV)}
    params = {k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param:")}
    model = HeteroSAGE(64, parallel.RELATIONS, num_layers=2).to(DEV)
    model.load_state_dict(params)
    pw = torch.from_numpy(z["pos_weights"]).to(DEV)
    shard = parallel.UserShard(ei, x["user"].shape[0], x["post"].shape[0], parallel.DistEnv(),
                               pos_weights=pw)
    h_u, h_p = shard.forward(model, x["user"], x["post"])
    close(h_u, z["out_user"])
    close(h_p, z["out_post"])
    loss = shard.loss(h_u, h_p, torch.from_numpy(z["neg_p"]).to(DEV))
    assert abs(float(loss.detach()) - float(z["loss"])) <= RTOL * abs(float(z["loss"]))
    loss.backward()
    grads = {name: p.grad.clone() for name, p in model.named_parameters()}
    for name, p in model.named_parameters():
        close(p.grad, z["grad:" + name])
        p.grad = None
    # the explicit schedule (UserShard.step): same kernels, same loss and gradients
    step_loss = shard.step(model, x["user"], x["post"], torch.from_numpy(z["neg_p"]).to(DEV))
    assert torch.equal(step_loss, loss.detach())
    for name, p in model.named_parameters():
        torch.testing.assert_close(p.grad, grads[name], rtol=1e-6, atol=1e-7)


def test_device_generated_graph_schema():
    cfg = synth.scaled("cfg2", 0.01)
    g = synth.make_graph(cfg, device=DEV, device_gen=True)
    e = g.edge_index_dict[synth.ENGAGES]
    assert e.shape == (2, cfg.num_engages) and e.dtype == torch.int64
    assert int(e[0].max()) < cfg.num_users and int(e[1].max()) < cfg.num_posts
    assert torch.equal(g.edge_index_dict[synth.REV_ENGAGES], e.flip(0))
    g2 = synth.make_graph(cfg, device=DEV, device_gen=True)
    assert torch.equal(g2.edge_index_dict[synth.ENGAGES], e)      # same on every rank


# ----------------------------------------------------------------------------- drop-in surface
def test_reference_structured_model_over_our_sageconv_matches_golden():
    """The reference's WeightedRGCN structure (train_gnn.py:147-200: three SAGEConv calls, torch
    weighted sum + ReLU) with only the import switched."""
    import torch.nn.functional as F

    class RefStructured(torch.nn.Module):
        def __init__(self, hidden_dim=64):
            super().__init__()
            self.msg_direct = SAGEConv((-1, -1), hidden_dim)
            self.msg_social = SAGEConv((-1, -1), hidden_dim)
            self.post_update = SAGEConv((-1, -1), hidden_dim)
            self.w_direct, self.w_social = 1.0, 0.75

        def forward(self, x_dict, edge_index_dict):
            u, p = x_dict["user"], x_dict["post"]
            md = self.msg_direct((p, u), edge_index_dict[("post", "rev_engages", "user")])
            ms = self.msg_social((u, u), edge_index_dict[("user", "social", "user")])
            uo = F.relu(self.w_direct * md + self.w_social * ms)
            po = F.relu(self.post_update((u, p), edge_index_dict[("user", "engages", "post")]))
            return {"user": uo, "post": po}

    z, x, e, params = _fixture_cfg1()
    model = RefStructured().to(DEV)
    model.load_state_dict(params)
    out = model(x, e)
    close(out["user"], z["out_user"])
    close(out["post"], z["out_post"])
    loss = ops.link_loss(out["user"], out["post"], e[synth.ENGAGES],
                         torch.from_numpy(z["neg_p"]).to(DEV),
                         torch.from_numpy(z["pos_weights"]).to(DEV))
    loss.backward()
    for name, p in model.named_parameters():
        close(p.grad, z["grad:" + name])


def test_integration_ctypes_snippet():
    """raw C ABI through ctypes, no torch types across the boundary."""
    import ctypes
    from truth_recommendation_gnn_amd import _native as Nn
    lib = ctypes.CDLL(str(Nn.LIB_PATH))
    P, I, L, S = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
    lib.hgnn_coo_to_csr_ws_bytes.restype = S
    lib.hgnn_coo_to_csr.argtypes = [P, P, L, L, L, P, P, P, P, P, S, P]
    lib.hgnn_gather_mean_fwd.argtypes = [P, L, I, P, P, L, P, P, L, L, I, P, P, P]
    p = lambda t: P(t.data_ptr()) if t is not None else None
    stream = P(torch.cuda.current_stream().cuda_stream)
    g = synth.make_graph("cfg1")
    ei = g.edge_index_dict[synth.REV_ENGAGES].to(DEV)
    src, dst = ei[0].contiguous(), ei[1].contiguous()
    x_src, n_dst = g.x_dict["post"].to(DEV), g.num_users
    E = src.numel()
    rowptr = torch.empty(n_dst + 1, dtype=torch.int32, device=DEV)
    col = torch.empty(E, dtype=torch.int32, device=DEV)
    perm = torch.empty(E, dtype=torch.int32, device=DEV)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    ws = torch.empty(lib.hgnn_coo_to_csr_ws_bytes(E, n_dst), dtype=torch.uint8, device=DEV)
    assert lib.hgnn_coo_to_csr(p(dst), p(src), E, n_dst, x_src.shape[0], p(rowptr), p(col),
                               p(perm), p(bad), p(ws), ws.numel(), stream) == 0
    aggr = torch.empty(n_dst, x_src.shape[1], device=DEV)
    assert lib.hgnn_gather_mean_fwd(p(x_src), x_src.shape[0], x_src.shape[1], p(rowptr), p(col),
                                    n_dst, None, None, 0, 0, 2**30, None, p(aggr), stream) == 0
    close(aggr, sage_ref.mean_aggregate(g.x_dict["post"], g.edge_index_dict[synth.REV_ENGAGES],
                                        n_dst))


# ----------------------------------------------------------------------------- pre-projection
@pytest.mark.parametrize("d", [64, 128])
def test_pre_projected_relation_matches_aggregate_first(monkeypatch, d):
    """Layer 2's post -> user relation projected on the (smaller) post table before the gather
    (ops.use_pre_projection) gives the aggregate-first result: outputs, fused loss and every
    parameter gradient, against each other and against the CPU oracle."""
    cfg = synth.dataclasses.replace(synth.scaled("cfg2", 0.002), dim=d, hidden=d)  # U=2000, P=200
    g = synth.make_graph(cfg)
    rels = [(synth.REV_ENGAGES, 1.0), (synth.ENGAGES, 1.0)]
    x = {k: v.to(DEV) for k, v in g.x_dict.items()}
    e = {k: v.to(DEV) for k, v in g.edge_index_dict.items()}
    pos = e[synth.ENGAGES]
    neg = synth.negative_posts(cfg.num_posts, pos.shape[1]).to(DEV)
    pw = synth.interaction_weights(cfg.num_posts).to(DEV)[pos[1]]
    torch.manual_seed(0)
    base = HeteroSAGE(d, rels, num_layers=2, in_channels=d).to(DEV)
    params = {k: v.detach().clone() for k, v in base.state_dict().items()}
    res = {}
    for pre in (False, True):
        monkeypatch.setattr(ops, "PRE_PROJECTION", pre)
        model = HeteroSAGE(d, rels, num_layers=2, in_channels=d).to(DEV)
        model.load_state_dict(params)
        out = model(x, e)
        loss = ops.edge_bce_loss(out["user"], out["post"], pos, neg, pw)
        loss.backward()
        res[pre] = (out, loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters()})
    (o0, l0, g0), (o1, l1, g1) = res[False], res[True]
    for t in ("user", "post"):
        close(o1[t], o0[t], rtol=1e-5)
    assert abs(float(l1) - float(l0)) <= 1e-6 * abs(float(l0))
    for n in g0:
        close(g1[n], g0[n], rtol=1e-5)
    # and the oracle (the reference's aggregate-then-project order)
    P = {k: v.cpu() for k, v in params.items()}
    ref_out, ref_loss, ref_grads = sage_ref.train_step_grads(
        P, lambda Q: sage_ref.hetero_sage(Q, g.x_dict, g.edge_index_dict, rels, 2),
        g.edge_index_dict[synth.ENGAGES], neg.cpu(), pw.cpu())
    for t in ("user", "post"):
        close(o1[t], ref_out[t])
    assert abs(float(l1) - float(ref_loss)) <= RTOL * abs(float(ref_loss))
    for n, r in ref_grads.items():
        close(g1[n], r)


def test_pre_projection_used_at_layer_two_only():
    """The rule on the bench's shapes: layer 1's static inputs keep aggregate-first (their
    projection gradient would need an extra K2 pass); layer 2's post table is projected."""
    x_post = torch.randn(100, 16, device=DEV)
    x_user = torch.randn(1000, 16, device=DEV)
    h_post = x_post.clone().requires_grad_()
    assert not ops.use_pre_projection(x_post, x_user, 16, True)        # layer 1, training
    assert ops.use_pre_projection(h_post, x_user, 16, True)            # layer 2
    assert not ops.use_pre_projection(x_user, x_post, 16, True)        # user -> post: bigger src
    assert not ops.use_pre_projection(h_post, x_user, 32, True)        # would widen the gather
    assert not ops.use_pre_projection(h_post, x_user, 16, False)       # no root segment
    with torch.no_grad():
        assert ops.use_pre_projection(x_post, x_user, 16, True)        # inference: always


def test_csr_cache_frees_structures_of_dead_edge_tensors():
    """100 edge tensors built and dropped (inference.py:410-419's per-user graphs, a per-step
    flip(0)): no cache entry and no device memory outlives them; a relation whose tensor died
    between forward and backward still back-propagates (its COO is rebuilt from the CSR, in the
    original edge order)."""
    import gc
    graph.CSR_CACHE.clear()
    gc.collect()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    rng = np.random.default_rng(3)
    for i in range(100):
        ei = rand_coo(rng, 300, 200, 2000 + i).to(DEV)
        csr = graph.relation_csr(ei, 300, 200)
        _ = csr.bwd, csr.inv_deg
        del ei, csr, _
    gc.collect()
    torch.cuda.synchronize()
    assert len(graph.CSR_CACHE) == 0
    assert torch.cuda.memory_allocated() == base
    # the tensor dies after the forward: the backward's CSC comes from the rebuilt COO
    x = torch.from_numpy(rng.standard_normal((300, 16)).astype(np.float32))
    ei_cpu = rand_coo(rng, 300, 200, 3000)
    xg = x.to(DEV).requires_grad_()
    ei = ei_cpu.to(DEV)
    csr = graph.relation_csr(ei, 300, 200)
    y = ops.mean_gather(xg, csr)
    del ei
    gc.collect()
    (y * y).sum().backward()
    xr = x.clone().requires_grad_()
    ref = sage_ref.mean_aggregate(xr, ei_cpu, 200)
    (ref * ref).sum().backward()
    close(y.detach().cpu(), ref.detach())
    close(xg.grad.cpu(), xr.grad)
    assert torch.equal(csr.edge_index.cpu(), ei_cpu)


# ----------------------------------------------------------------------------- K3 on both paths
@contextlib.contextmanager
def _k3_split(on):
    """K3 at H = 128, K = 128 / 256: the bf16x6 split (True, the default) or the f32-input MFMA
    kernels (False)."""
    from truth_recommendation_gnn_amd import _native as N
    prev = N.lib().hgnn_set_k3_split(int(on))
    try:
        yield
    finally:
        N.lib().hgnn_set_k3_split(prev)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("ks", [[128], [128, 128], [64, 64, 128], [64, 64], [128, 128, 128],
                                [64, 256, 64]])
def test_linear_h128_on_both_k3_paths(split, ks):
    """The H = 128 shapes the split covers (K = 128 and 256, 128-column segments and others;
    K = 384 / 512 as two column blocks, a segment straddling the block edge included),
    through forward (with the added input and the ReLU bits), every backward mode and the
    accumulating dX, on the split and on the f32-input MFMA kernels it replaces by default."""
    with _k3_split(split):
        for n in (37, 20000):
            test_linear_fwd_bwd_matches_torch(ks, 128, n)
        for mode in ("no_relu", "dx_subset", "wgrad_only", "db_only", "dgrad_only"):
            test_linear_bwd_variants(ks, 128, mode)
        for masked in (False, True):
            test_linear_bwd_dx_accumulate_bitwise(ks, 128, masked)
        for mode in ("all", "wgrad_only", "dz_out"):
            test_linear_relu_bits_equal_float_mask(ks, 128, mode)


@pytest.mark.parametrize("ks", [[128], [128, 128]])
@pytest.mark.parametrize("relu", [False, True])
def test_linear_split_passes_inf_and_nan_like_f32_kernels(ks, relu):
    """Non-finite inputs: an inf or NaN in X gives the split the +-inf / NaN pattern
    of the f32-input kernels in the forward, and an inf in dout the same dX, rather than NaN
    from inf - bf16(inf) in a residual piece or from inf times W's mixed-sign residual pieces."""
    gen = torch.Generator().manual_seed(7)
    n, K = 300, sum(ks)
    segs = [torch.randn(n, k, generator=gen) for k in ks]
    segs[0][5, 3] = float("inf")
    segs[-1][9, 17] = float("-inf")
    segs[0][11, 40] = float("nan")
    w = torch.randn(128, K, generator=gen) * 0.1
    b = torch.randn(128, generator=gen)
    dout = torch.randn(n, 128, generator=gen)
    dout[20, 7] = float("inf")
    dout[21, 9] = float("-inf")
    res = {}
    for split in (False, True):
        with _k3_split(split):
            sd = [s_.to(DEV) for s_ in segs]
            out = ops.linear_fwd(sd, w.to(DEV), b.to(DEV), relu)
            dxs = [torch.empty_like(s_) for s_ in sd]
            finite = [s_.nan_to_num(0.0, 0.0, 0.0) for s_ in sd]
            ops.linear_bwd(finite, w.to(DEV), dout.to(DEV), None, dxs, False, False)
            res[split] = (out.cpu(), torch.cat([d.cpu() for d in dxs], 1))
    for a, c in zip(res[False], res[True]):
        assert torch.equal(torch.isnan(a), torch.isnan(c))
        assert torch.equal(torch.isposinf(a), torch.isposinf(c))
        assert torch.equal(torch.isneginf(a), torch.isneginf(c))
        fin = torch.isfinite(a)
        assert bool(torch.isinf(a).any()) or relu
        scale = float(a[fin].abs().max())
        assert float((a[fin] - c[fin]).abs().max()) <= 2e-5 * scale


@pytest.mark.parametrize("ks", [[128, 128, 128], [128, 128, 128, 128]])
def test_k3_split_wide_matches_f32_kernels_closely(ks):
    """K = 384 / 512 (cfg5's sampled blocks: [aggr_1 | aggr_2 | root]) on the split as two column
    blocks — the second launch adding the first one's output rows, dW reduced per column block —
    against the f32-input general kernels, at a block-sized row count: within 2e-5 of each
    tensor's max."""
    gen = torch.Generator().manual_seed(13)
    n = 17_003
    segs = [torch.randn(n, k, generator=gen).to(DEV) for k in ks]
    w = (torch.randn(128, sum(ks), generator=gen) * 0.1).to(DEV)
    b = torch.randn(128, generator=gen).to(DEV)
    add = torch.randn(n, 128, generator=gen).to(DEV)
    dout = torch.randn(n, 128, generator=gen).to(DEV)
    res = {}
    for split in (False, True):
        with _k3_split(split):
            mk = ops.relu_mask_for(n, 128, True, torch.device(DEV))
            out = ops.linear_fwd(segs, w, b, True, add=add, mask_out=mk)
            dxs = [torch.empty_like(s) for s in segs]
            dw, db = ops.linear_bwd(segs, w, dout, out, dxs, True, True, mask=mk)
            res[split] = [out, *dxs, dw, db]
    for a, c in zip(res[False], res[True]):
        scale = float(a.abs().max())
        assert float((a - c).abs().max()) <= 2e-5 * scale, (float((a - c).abs().max()), scale)


def test_k3_split_matches_f32_kernels_closely():
    """At a cfg4-like K = 256 shape the split and the f32-input kernels agree to fp32 rounding:
    forward outputs, dX, dW, db within 2e-5 of each tensor's max (dW / db sum 50k rows in
    different tile orders on the two paths)."""
    gen = torch.Generator().manual_seed(11)
    n = 50_000
    segs = [torch.randn(n, 128, generator=gen).to(DEV) for _ in range(2)]
    w = (torch.randn(128, 256, generator=gen) * 0.1).to(DEV)
    b = torch.randn(128, generator=gen).to(DEV)
    dout = torch.randn(n, 128, generator=gen).to(DEV)
    res = {}
    for split in (False, True):
        with _k3_split(split):
            out = ops.linear_fwd(segs, w, b, True)
            dxs = [torch.empty_like(s) for s in segs]
            dw, db = ops.linear_bwd(segs, w, dout, out, dxs, True, True)
            res[split] = [out, *dxs, dw, db]
    for a, c in zip(res[False], res[True]):
        scale = float(a.abs().max())
        assert float((a - c).abs().max()) <= 2e-5 * scale, (float((a - c).abs().max()), scale)


@pytest.mark.parametrize("d", [128, 64, 16])
def test_gather_multi_equals_single_calls(d):
    """hgnn_gather_reduce_multi (a sampled layer's K1s, or one round of its K2s, as one launch;
    round 6) against one hgnn_gather_reduce per job: the mean gathers into fresh outputs and the
    weighted K2s accumulating into existing ones, bitwise; empty rows and an empty relation
    included."""
    from truth_recommendation_gnn_amd import graph as G
    gen = torch.Generator().manual_seed(d)
    jobs = []
    for n_dst, n_src, max_deg in [(300, 50, 6), (100, 700, 12), (0, 10, 0), (257, 257, 3)]:
        deg = torch.randint(0, max_deg + 1, (n_dst,), generator=gen)
        rowptr = torch.zeros(n_dst + 1, dtype=torch.int32)
        rowptr[1:] = torch.cumsum(deg, 0)
        col = torch.randint(0, n_src, (int(rowptr[-1]),), generator=gen, dtype=torch.int32)
        csr = G.RelationCSR.from_csr(rowptr.to(DEV), col.to(DEV), n_src, n_dst,
                                     may_have_heavy_rows=False)
        x = torch.randn(n_src, d, generator=gen).to(DEV)
        jobs.append((x, csr))
    got = ops.gather_mean_many(jobs)
    for (x, csr), o in zip(jobs, got):
        assert torch.equal(o, ops.gather_mean(x, csr))
    # K2 round: accumulate into per-job outputs with the CSC weights
    outs = [torch.randn(csr.n_src, d, generator=gen).to(DEV) for _, csr in jobs]
    dAs = [torch.randn(csr.n_dst, d, generator=gen).to(DEV) for _, csr in jobs]
    ref = [o.clone() for o in outs]
    for dA, (_, csr), r in zip(dAs, jobs, ref):
        ops.scatter_mean_bwd(dA, csr, out=r)
    ops._gather_multi([(dA, csr.bwd, o) for dA, (_, csr), o in zip(dAs, jobs, outs)],
                      mean=False, accumulate=True, edge_ws=[c.bwd_weights for _, c in jobs])
    for o, r in zip(outs, ref):
        assert torch.equal(o, r)


@pytest.mark.parametrize("case", ["pair", "pair_root", "small", "k_differs", "w_differs"])
def test_linear_multi_equals_per_job_calls(case):
    """hgnn_linear_fwd_multi / hgnn_linear_bwd_multi (a sampled layer's two destination types'
    K3 as one launch per column block, round 6) against one hgnn_linear_fwd_mask /
    hgnn_linear_bwd_ex call per job.  The forward's rows, the ReLU bits and dX do not depend on
    the grid: bitwise.  dW / db are the same partial sums over a different block split (the pair
    shares one chip's worth of blocks): within 2e-6 of the largest entry.  'k_differs' (K = 384
    beside K = 512) and 'w_differs' (one job without weight gradients: a different kernel
    variant) run job by job: bitwise throughout."""
    gen = torch.Generator().manual_seed(7)
    h = 128
    shapes = {"pair": [(9000, [128, 128, 128]), (12345, [128, 128, 128])],
              "pair_root": [(8192, [128, 128, 128]), (20000, [128, 128, 128])],
              "k_differs": [(9000, [128, 128, 128]), (10000, [128, 128, 128, 128])],
              "small": [(3000, [128, 128, 128]), (2500, [128, 128, 128])],
              "w_differs": [(9000, [128, 128, 128]), (7000, [128, 128, 128])]}[case]
    jobs_f, ref_f = [], []
    for n, ks in shapes:
        segs = [torch.randn(n, k, generator=gen).to(DEV) for k in ks]
        w = (torch.randn(h, sum(ks), generator=gen) * 0.05).to(DEV)
        b = torch.randn(h, generator=gen).to(DEV)
        mk = ops.relu_mask_for(n, h, True, torch.device(DEV), sum(ks))
        jobs_f.append((segs, w, b, True, mk))
        mk_ref = None if mk is None else torch.empty_like(mk)
        ref_f.append((ops.linear_fwd(segs, w, b, True, mask_out=mk_ref), mk_ref))
    outs = ops.linear_fwd_many(jobs_f)
    for o, (r, mr), (_, _, _, _, mk) in zip(outs, ref_f, jobs_f):
        assert torch.equal(o, r)
        if mk is not None:
            assert torch.equal(mk, mr)
    # backward: dX of the first two segments; the root segment's dX only in 'pair_acc_root'
    jobs_b, ref_b = [], []
    for i, ((segs, w, b, _, mk), o) in enumerate(zip(jobs_f, outs)):
        dout = torch.randn(o.shape, generator=gen).to(DEV)
        root = case == "pair_root"
        dxs = [torch.empty_like(s_) for s_ in segs[:2]] + \
            [torch.empty_like(s_) if root else None for s_ in segs[2:]]
        dxs_ref = [None if d is None else torch.empty_like(d) for d in dxs]
        need = not (case == "w_differs" and i == 1)
        jobs_b.append((segs, w, dout, o, dxs, need, need, mk))
        ref_b.append((ops.linear_bwd(segs, w, dout, o, dxs_ref, need, need, mask=mk), dxs_ref))
    got = ops.linear_bwd_many(jobs_b)
    for (dw, db), ((rdw, rdb), dxs_ref), job in zip(got, ref_b, jobs_b):
        for d, r in zip(job[4], dxs_ref):
            if d is not None:
                assert torch.equal(d, r)
        exact = case in ("k_differs", "w_differs")
        for a, r in ((dw, rdw), (db, rdb)):
            if r is None:
                assert a is None
            elif exact:
                assert torch.equal(a, r)
            else:
                tol = 2e-6 * float(r.abs().max())
                assert float((a - r).abs().max()) <= tol, (float((a - r).abs().max()), tol)


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_adam_matches_torch(wd):
    """optim.Adam (hgnn_adam_multi: every parameter in one launch, the step count on the device)
    against torch.optim.Adam(fused=True) over 6 steps with the same gradients: 40 tensors (two
    launches of 32), odd sizes, an empty one; then a recorded step replayed 3 times against 3
    eager steps, bitwise, and the device step count."""
    from truth_recommendation_gnn_amd import optim
    gen = torch.Generator().manual_seed(11)
    shapes = [(128, 384), (128,), (7,), (0,), (33, 5)] * 8
    init = [torch.randn(s, generator=gen) for s in shapes]
    ours = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    ref = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    opt = optim.Adam(ours, lr=1e-3, weight_decay=wd)
    opt_ref = torch.optim.Adam(ref, lr=1e-3, weight_decay=wd, fused=True)
    for _ in range(6):
        grads = [torch.randn(s, generator=gen).to(DEV) for s in shapes]
        for p, q, g in zip(ours, ref, grads):
            p.grad = g.clone()
            q.grad = g.clone()
        opt.step()
        opt_ref.step()
    assert opt.steps_done() == 6
    worst = 0.0
    for p, q in zip(ours, ref):
        if p.numel():
            worst = max(worst, float((p - q).abs().max() / q.abs().max().clamp_min(1e-30)))
    assert worst <= 1e-6, worst
    # recorded: one eager step done above; capture one step and replay it 3 times
    twin = [torch.nn.Parameter(p.detach().clone()) for p in ours]
    opt_twin = optim.Adam(twin, lr=1e-3, weight_decay=wd)
    for p, q in zip(ours, twin):
        q.grad = p.grad.clone()
    opt_twin.step()                                    # the twin's state: 1 step
    for p, q in zip(ours, twin):                      # ours: 6 steps; restart both from equal
        q.data.copy_(p.data)
        opt_twin.state[q]["exp_avg"].copy_(opt.state[p]["exp_avg"])
        opt_twin.state[q]["exp_avg_sq"].copy_(opt.state[p]["exp_avg_sq"])
    opt_twin.param_groups[0]["_dev_state"][0].fill_(6.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            opt_twin.step()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        grads = [torch.randn(sh, generator=gen).to(DEV) for sh in shapes]
        for p, q, gr in zip(ours, twin, grads):
            p.grad.copy_(gr)
            q.grad.copy_(gr)
        opt.step()
        g.replay()
    torch.cuda.synchronize()
    assert opt.steps_done() == 9 and opt_twin.steps_done() == 9
    for p, q in zip(ours, twin):
        assert torch.equal(p, q)
