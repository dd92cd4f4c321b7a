"""The captured mini-batch step (minibatch.py: static-capacity blocks replayed as one HIP graph)
against the eager step on the same sampled batches (sampler.forward_blocks, itself checked
against plain torch on the blocks in test_sampler.py): seed outputs, loss and every parameter
gradient, then whole Adam training steps.  Plus the padding kernel's invariants."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _csr(rng, n_dst, n_src, max_deg):
    deg = rng.integers(0, max_deg + 1, n_dst)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    col = rng.integers(0, n_src, int(rowptr[-1])).astype(np.int32)
    return torch.from_numpy(rowptr).to(DEV), torch.from_numpy(col).to(DEV)


def test_pad_csr_multi_keeps_real_rows_and_spreads_padding():
    from truth_recommendation_gnn_amd import _native as N
    rng = np.random.default_rng(3)
    items = []
    for n_dst, n_src, max_deg, d_cap, e_cap, mapped in [(300, 50, 6, 340, 2000, False),
                                                        (100, 70, 3, 101, 400, True),
                                                        (0, 10, 0, 16, 64, False),
                                                        (64, 64, 5, 64 + 1, 64 * 5, False)]:
        rp, col = _csr(rng, n_dst, n_src, max_deg)
        mp = torch.from_numpy(rng.permutation(10_000)[:n_src].astype(np.int32)).to(DEV) \
            if mapped else None
        items.append((rp, col, mp, n_dst, int(col.numel()), d_cap, e_cap, 7))
    ids = torch.arange(5, 25, dtype=torch.int32, device=DEV)
    outs = [(torch.full((it[5] + 1,), -9, dtype=torch.int32, device=DEV),
             torch.full((it[6],), -9, dtype=torch.int32, device=DEV)) for it in items]
    ids_out = torch.full((32,), -9, dtype=torch.int32, device=DEV)
    n = len(items) + 1
    N.check(N.lib().hgnn_pad_csr_multi(
        n, N.ptr_array([it[0] for it in items] + [None]),
        N.ptr_array([it[1] if it[4] else None for it in items] + [ids]),
        N.ptr_array([it[2] for it in items] + [None]),
        N.i64_array([it[3] for it in items] + [0]), N.i64_array([it[4] for it in items] + [20]),
        N.ptr_array([o[0] for o in outs] + [None]), N.ptr_array([o[1] for o in outs] + [ids_out]),
        N.i64_array([it[5] for it in items] + [-1]), N.i64_array([it[6] for it in items] + [32]),
        N.int_array([it[7] for it in items] + [0]), N.int_array([1, 3, 1, 2, 1]),
        N.stream_ptr(DEV)), "pad")
    for (rp, col, mp, n_dst, E, d_cap, e_cap, dummy), (rpo, colo), spread in zip(items, outs,
                                                                                 [1, 3, 1, 2]):
        rpo, colo = rpo.cpu(), colo.cpu()
        assert torch.equal(rpo[:n_dst + 1], rp.cpu())                 # real rows untouched
        assert int(rpo[-1]) == e_cap and bool((rpo[1:] >= rpo[:-1]).all())
        want = col.cpu().long() if mp is None else mp.cpu()[col.cpu().long()]
        assert torch.equal(colo[:E].long(), want.long())
        assert torch.equal(colo[E:].long(), dummy + torch.arange(e_cap - E) % spread)
        lens = (rpo[n_dst + 1:] - rpo[n_dst:-1]).numpy()                 # padded rows balanced
        assert lens.sum() == e_cap - E and lens.max() - lens.min() <= 1
    assert ids_out[:20].tolist() == list(range(5, 25)) and ids_out[20:].eq(0).all()
    # a batch larger than the capacity is refused, not written out of bounds
    rp, col = _csr(rng, 10, 5, 4)
    with pytest.raises(N.NativeError, match="capacity"):
        N.check(N.lib().hgnn_pad_csr_multi(
            1, N.ptr_array([rp]), N.ptr_array([col]), N.ptr_array([None]), N.i64_array([10]),
            N.i64_array([int(col.numel())]), N.ptr_array([outs[0][0]]),
            N.ptr_array([outs[0][1]]), N.i64_array([10]), N.i64_array([400]),
            N.int_array([0]), None, N.stream_ptr(DEV)), "pad")


def _setup(seed_n=24, fanouts=(5, 3)):
    from truth_recommendation_gnn_amd import HeteroSAGE, sampler, synth
    cfg = synth.dataclasses.replace(synth.scaled("cfg5", 0.0002), dim=16, hidden=16)
    g = synth.make_graph(cfg, device=DEV)
    rels = [(synth.REV_ENGAGES, 1.0), (synth.SOCIAL, 0.75), (synth.ENGAGES, 1.0),
            (synth.POST_POST, 0.5)]
    num = {"user": cfg.num_users, "post": cfg.num_posts}
    s = sampler.NeighborSampler(num, g.edge_index_dict, [et for et, _ in rels], list(fanouts))
    gen = torch.Generator(device=DEV).manual_seed(1)
    order = {"user": torch.randperm(cfg.num_users, device=DEV, generator=gen),
             "post": torch.randperm(cfg.num_posts, device=DEV, generator=gen)}

    def batch(b):
        return s.sample({t: o[b * seed_n:(b + 1) * seed_n] for t, o in order.items()}, seed=b)

    def make_model():
        torch.manual_seed(synth.WEIGHT_SEED)
        return HeteroSAGE(cfg.hidden, rels, num_layers=2, in_channels=cfg.dim).to(DEV)

    return g, s, batch, make_model, {"user": seed_n, "post": seed_n}


def _loss(out):
    u, p = out["user"], out["post"]
    pos = (u * p).sum(1)
    neg = (u * p.roll(1, 0)).sum(1)
    return torch.nn.functional.softplus(-pos).mean() + torch.nn.functional.softplus(neg).mean()


def _close(got, ref, what):
    scale = float(ref.abs().max())
    err = float((got - ref).abs().max()) / max(scale, 1e-30)
    assert err < 1e-4, (what, err)


def test_captured_step_matches_eager_blocks():
    """Forward + loss + backward on static blocks, replayed for new batches, against the eager
    block step on the same batches: seed outputs, loss and every gradient (rtol 1e-4 of each
    tensor's max; the padded rows only change the order of fp32 sums in the weight gradients)."""
    from truth_recommendation_gnn_amd import minibatch, sampler
    g, s, batch, make_model, n_seeds = _setup()
    model = make_model()
    step = minibatch.CapturedStep(model, g.x_dict, s, n_seeds, _loss, None, slack=16)
    step.capture(batch(0))
    caps = step.blocks.cap
    for b in (1, 2, 5):
        mb = batch(b)
        # the batch fits the static layout with room to spare (the slack rows stay padding)
        for h, blk in enumerate(mb.blocks[::-1]):
            for t, n in blk.n_dst.items():
                assert n <= caps[h][t] - 16
        loss = step.step(mb)
        got_out = {t: v.detach().clone() for t, v in step.out.items()}
        got_loss = float(loss)
        got = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
        ref_model = make_model()
        ref_model.load_state_dict(model.state_dict())
        out = sampler.forward_blocks(ref_model, mb, g.x_dict)
        ref_loss = _loss(out)
        ref_loss.backward()
        for t in out:
            _close(got_out[t], out[t].detach(), f"out {t}")
        assert abs(got_loss - float(ref_loss)) <= 1e-5 * abs(float(ref_loss)), (got_loss, ref_loss)
        for n, p in ref_model.named_parameters():
            _close(got[n], p.grad, n)


def test_captured_adam_steps_match_eager_training():
    """Whole training steps (forward, loss, backward, Adam) replayed from the graph against the
    same steps run eagerly from the same initial weights: the capture's own warm-up steps (on
    the first batch) and then one replay per batch."""
    from truth_recommendation_gnn_amd import minibatch, sampler
    g, s, batch, make_model, n_seeds = _setup()
    model, ref = make_model(), make_model()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True, capturable=True)
    ref_opt = torch.optim.Adam(ref.parameters(), lr=1e-3, fused=True)
    step = minibatch.CapturedStep(model, g.x_dict, s, n_seeds, _loss, opt, slack=16)
    step.capture(batch(0), warmup=2)
    for b in (0, 0):                                  # the eager twin of the warm-up steps
        ref_opt.zero_grad(set_to_none=True)
        _loss(sampler.forward_blocks(ref, batch(b), g.x_dict)).backward()
        ref_opt.step()
    for b in (1, 2, 3):
        step.step(batch(b))
        ref_opt.zero_grad(set_to_none=True)
        _loss(sampler.forward_blocks(ref, batch(b), g.x_dict)).backward()
        ref_opt.step()
    torch.cuda.synchronize()
    for (n, p), (_, r) in zip(model.named_parameters(), ref.named_parameters()):
        _close(p.detach(), r.detach(), n)
        assert not torch.equal(p.detach(), make_model().state_dict()[n])   # it trained


@pytest.mark.parametrize("case", ["one_layer", "one_relation"])
def test_captured_step_layouts(case):
    """One layer (the outermost block is also the seeds' block), and a single relation (posts
    have no incoming relation: their rows pass through as roots); plus the seed-count guard."""
    from truth_recommendation_gnn_amd import HeteroSAGE, minibatch, sampler, synth
    cfg = synth.dataclasses.replace(synth.scaled("cfg5", 0.0002), dim=16, hidden=16)
    g = synth.make_graph(cfg, device=DEV)
    rels = ([(synth.REV_ENGAGES, 1.0), (synth.SOCIAL, 0.75), (synth.ENGAGES, 1.0)]
            if case == "one_layer" else [(synth.REV_ENGAGES, 1.0)])
    layers, fanouts = (1, [6]) if case == "one_layer" else (2, [4, 2])
    num = {"user": cfg.num_users, "post": cfg.num_posts}
    s = sampler.NeighborSampler(num, g.edge_index_dict, [et for et, _ in rels], fanouts)
    n = 20
    seeds = lambda b: {"user": torch.arange(b * n, (b + 1) * n, device=DEV),   # noqa: E731
                       "post": torch.arange(b * n, (b + 1) * n, device=DEV)}
    torch.manual_seed(3)
    model = HeteroSAGE(cfg.hidden, rels, num_layers=layers, in_channels=cfg.dim).to(DEV)
    step = minibatch.CapturedStep(model, g.x_dict, s, {"user": n, "post": n}, _loss, None, slack=8)
    step.capture(s.sample(seeds(0), seed=0))
    mb = s.sample(seeds(3), seed=3)
    got_loss = float(step.step(mb))
    got = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    model.zero_grad(set_to_none=True)
    ref = _loss(sampler.forward_blocks(model, mb, g.x_dict))
    ref.backward()
    assert abs(got_loss - float(ref)) <= 1e-5 * abs(float(ref))
    for k, p in model.named_parameters():
        if p.grad is not None:
            _close(got[k], p.grad, k)
    with pytest.raises(ValueError, match="exceed"):
        step.step(s.sample({"user": torch.arange(n + 1, device=DEV),
                            "post": torch.arange(n, device=DEV)}))
    # a short batch would feed padded rows to this loss (it reads every seed row): refused
    # unless the loss reads rows by id (LinkLoss sets partial_seeds)
    assert not step.blocks.partial_seeds
    with pytest.raises(ValueError, match="partial_seeds"):
        step.step(s.sample({"user": torch.arange(n - 1, device=DEV),
                            "post": torch.arange(n, device=DEV)}))


# ----------------------------------------------------------------------------- link batches (cfg5)
def _link_setup(B=48, fanouts=(5, 3)):
    from truth_recommendation_gnn_amd import minibatch, synth
    g, s, _, make_model, _ = _setup(fanouts=fanouts)
    ei = g.edge_index_dict[synth.ENGAGES]
    P = g.x_dict["post"].shape[0]
    gen = torch.Generator(device=DEV).manual_seed(5)
    order = torch.randperm(int(ei.shape[1]), device=DEV, generator=gen)

    def batch(b):
        lb = minibatch.link_batch(ei, order[b * B:(b + 1) * B], int(P), generator=gen)
        lb.mb = s.sample(lb.seeds, seed=b)
        return lb
    return g, s, batch, make_model, ei, int(P), {"user": B, "post": 2 * B}


def test_link_batch_positives_are_graph_edges():
    """cfg5's batches are link prediction on real edges: every positive pair is an
    engages edge of the graph, the negatives are posts, the seeds are the distinct endpoints
    (sorted), and the local ids index the seeds (= the sampled outputs' rows)."""
    g, s, batch, _, ei, P, _ = _link_setup()
    U = int(g.x_dict["user"].shape[0])
    keys = ei[0].long() * P + ei[1].long()
    for b in (0, 1, 7):
        lb = batch(b)
        assert bool(torch.isin(lb.pos_u.long() * P + lb.pos_p.long(), keys).all())
        assert int(lb.neg_p.min()) >= 0 and int(lb.neg_p.max()) < P
        for t, n_max in (("user", U), ("post", P)):
            sd = lb.seeds[t]
            assert bool((sd[1:] > sd[:-1]).all()) and int(sd.max()) < n_max
        assert torch.equal(lb.seeds["user"][lb.pu], lb.pos_u)
        assert torch.equal(lb.seeds["post"][lb.pp], lb.pos_p)
        assert torch.equal(lb.seeds["post"][lb.pn], lb.neg_p)
        assert torch.equal(lb.mb.nodes[-1]["user"].long(), lb.seeds["user"])


def _ref_link_loss(out, lb):
    """The reference's loss on the batch's pairs (train_gnn.py:259-281, unit edge weights)."""
    u, p = out["user"], out["post"]
    pos = (u[lb.pu] * p[lb.pp]).sum(1)
    neg = (u[lb.pu] * p[lb.pn]).sum(1)
    return (torch.nn.functional.softplus(-pos).mean()
            + torch.nn.functional.softplus(neg).mean())


def test_captured_link_step_matches_reference_loss():
    """The captured link-prediction step (static capacities: B users, 2B posts; the fused loss
    over the pairs, its groupings staged before the replay) against the eager block forward
    with the reference loss as torch ops, on new batches: loss and every gradient."""
    from truth_recommendation_gnn_amd import minibatch, sampler
    g, s, batch, make_model, _, _, n_seeds = _link_setup()
    B = n_seeds["user"]
    model = make_model()
    ll = minibatch.LinkLoss(B, n_seeds["user"], n_seeds["post"], DEV)
    step = minibatch.CapturedStep(model, g.x_dict, s, n_seeds, ll, None, slack=16)
    assert step.blocks.partial_seeds              # LinkLoss reads seed rows by local id
    lb0 = batch(0)
    ll.load(lb0.pu, lb0.pp, lb0.pn)
    step.capture(lb0.mb)
    nodes = step.graph_nodes()                    # the recorded step, by node kind
    assert nodes["kernel"] >= 15 and nodes["total"] == sum(
        nodes[k] for k in ("kernel", "memcpy", "memset", "other"))
    for b in (1, 2, 6):
        lb = batch(b)
        ll.load(lb.pu, lb.pp, lb.pn)
        got_loss = float(step.step(lb.mb))
        got = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
        ref_model = make_model()
        ref_model.load_state_dict(model.state_dict())
        ref = _ref_link_loss(sampler.forward_blocks(ref_model, lb.mb, g.x_dict), lb)
        ref.backward()
        assert abs(got_loss - float(ref)) <= 2e-6 * abs(float(ref)), (got_loss, float(ref))
        for n, p in ref_model.named_parameters():
            _close(got[n], p.grad, n)


def test_captured_link_step_with_gradient_hook_trains_like_eager():
    """The data-parallel form of the captured step: forward + loss + backward replayed, an eager
    hook on the gradients (parallel.sync_grads' all-reduce at N > 1; here a stand-in that scales
    them), then the replayed Adam step — against the same training steps run eagerly."""
    from truth_recommendation_gnn_amd import minibatch, sampler
    g, s, batch, make_model, _, _, n_seeds = _link_setup()
    B = n_seeds["user"]
    model, ref = make_model(), make_model()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True, capturable=True)
    ref_opt = torch.optim.Adam(ref.parameters(), lr=1e-3, fused=True)

    def hook(m):
        for p in m.parameters():
            if p.grad is not None:
                p.grad.mul_(0.5)
    ll = minibatch.LinkLoss(B, n_seeds["user"], n_seeds["post"], DEV)
    step = minibatch.CapturedStep(model, g.x_dict, s, n_seeds, ll, opt, slack=16,
                                  between=lambda: hook(model))
    lb0 = batch(0)
    ll.load(lb0.pu, lb0.pp, lb0.pn)
    step.capture(lb0.mb, warmup=2)
    assert step.graph_opt is not None
    losses = []
    for lb in [lb0, lb0] + [batch(b) for b in (1, 2, 3)]:
        if lb is not lb0:
            ll.load(lb.pu, lb.pp, lb.pn)
            losses.append(float(step.step(lb.mb)))
        ref_opt.zero_grad(set_to_none=True)
        _ref_link_loss(sampler.forward_blocks(ref, lb.mb, g.x_dict), lb).backward()
        hook(ref)
        ref_opt.step()
    torch.cuda.synchronize()
    for (n, p), (_, r) in zip(model.named_parameters(), ref.named_parameters()):
        _close(p.detach(), r.detach(), n)
    assert all(np.isfinite(losses))


def test_captured_link_step_with_rccl_allreduce_in_the_graph():
    """over RCCL the data-parallel step is ONE replay — forward + loss + backward,
    parallel.sync_grads' flat all-reduce (issued at world 1 too: force=True) and the Adam step
    recorded in one HIP graph — and it trains like the eager steps (an all-reduce over one rank
    is the identity; the hook's scaling inside the graph shows the recorded call runs)."""
    import os
    import socket
    import torch.distributed as dist
    from truth_recommendation_gnn_amd import minibatch, parallel, sampler
    if dist.is_initialized():
        pytest.skip("a process group is already up in this process")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1)
    step = None
    try:
        env = parallel.DistEnv.from_torch()
        g, s, batch, make_model, _, _, n_seeds = _link_setup()
        B = n_seeds["user"]
        model, ref = make_model(), make_model()
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True, capturable=True)
        ref_opt = torch.optim.Adam(ref.parameters(), lr=1e-3, fused=True)

        def hook(m):
            for p in m.parameters():
                if p.grad is not None:
                    p.grad.mul_(0.5)

        def between():
            parallel.sync_grads(model, env, force=True)
            hook(model)
        ll = minibatch.LinkLoss(B, n_seeds["user"], n_seeds["post"], DEV)
        step = minibatch.CapturedStep(model, g.x_dict, s, n_seeds, ll, opt, slack=16,
                                      between=between, capture_between=True)
        lb0 = batch(0)
        ll.load(lb0.pu, lb0.pp, lb0.pn)
        step.capture(lb0.mb, warmup=2)
        assert step.graph_opt is None               # one graph: the collective is inside it
        losses = []
        for lb in [lb0, lb0] + [batch(b) for b in (1, 2, 3)]:
            if lb is not lb0:
                ll.load(lb.pu, lb.pp, lb.pn)
                losses.append(float(step.step(lb.mb)))
            ref_opt.zero_grad(set_to_none=True)
            _ref_link_loss(sampler.forward_blocks(ref, lb.mb, g.x_dict), lb).backward()
            hook(ref)
            ref_opt.step()
        torch.cuda.synchronize()
        for (n, p), (_, r) in zip(model.named_parameters(), ref.named_parameters()):
            _close(p.detach(), r.detach(), n)
        assert all(np.isfinite(losses))
    finally:
        # the recorded graphs hold the communicator's collective: release them (and let the
        # GPU drain) before the process group goes (its teardown aborted with them alive)
        del step
        import gc
        gc.collect()
        torch.cuda.synchronize()
        dist.destroy_process_group()


def test_captured_link_step_prepared_on_a_side_stream():
    """The bench's pipeline (round 6): each batch is sampled and prepared — padded blocks, root
    rows, the inner blocks' CSCs, the loss's groupings — into the staging buffers on a side
    stream while the previous replay runs, then committed (one copy) and replayed: loss and
    every gradient as the eager step with the reference loss on the same batch."""
    from truth_recommendation_gnn_amd import minibatch, sampler
    g, s, batch, make_model, _, _, n_seeds = _link_setup()
    B = n_seeds["user"]
    model = make_model()
    ll = minibatch.LinkLoss(B, n_seeds["user"], n_seeds["post"], DEV)
    step = minibatch.CapturedStep(model, g.x_dict, s, n_seeds, ll, None, slack=16)
    lb0 = batch(0)
    ll.load(lb0.pu, lb0.pp, lb0.pn)
    step.capture(lb0.mb)
    main, side = torch.cuda.current_stream(DEV), torch.cuda.Stream(DEV)
    lbs = {}

    def prep(b):
        side.wait_stream(main)
        with torch.cuda.stream(side):
            lbs[b] = lb = batch(b)
            step.prepare(lb.mb, lb.pu, lb.pp, lb.pn)
    prep(1)
    for b in (1, 2, 3):
        main.wait_stream(side)
        loss = step.step()                  # commits what prep(b) staged
        prep(b + 1)                         # the next batch, under this replay
        got_loss = float(loss)
        got = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
        torch.cuda.synchronize()
        ref_model = make_model()
        ref_model.load_state_dict(model.state_dict())
        ref = _ref_link_loss(sampler.forward_blocks(ref_model, lbs[b].mb, g.x_dict), lbs[b])
        ref.backward()
        assert abs(got_loss - float(ref)) <= 2e-6 * abs(float(ref)), (b, got_loss, float(ref))
        for n, p in ref_model.named_parameters():
            _close(got[n], p.grad, n)


def test_link_sampler_stages_what_the_eager_sampler_stages():
    """The sync-free LinkSampler (round 6: device-side counts, no read-back) against link_batch
    + NeighborSampler.sample + CapturedStep.prepare on the same edges, draws and seed: every
    staged byte — padded block CSRs, root ids and rows, the inner CSCs and 1/deg, the loss
    groupings — equal, and the sampled edge count equal; then a replay on it gives the reference
    loss."""
    from truth_recommendation_gnn_amd import minibatch, sampler
    g, s, _, make_model, ei, P, n_seeds = _link_setup()
    B = n_seeds["user"]
    model = make_model()
    ll = minibatch.LinkLoss(B, n_seeds["user"], n_seeds["post"], DEV)
    step = minibatch.CapturedStep(model, g.x_dict, s, n_seeds, ll, None, slack=16)
    ls = minibatch.LinkSampler(step, ei, P)
    order = torch.randperm(int(ei.shape[1]), device=DEV,
                           generator=torch.Generator(device=DEV).manual_seed(7))
    barena, larena = step.blocks.arena._bytes["stage"], ll.arena._bytes["stage"]
    for b in range(4):
        ids = order[b * B:(b + 1) * B]
        lb = minibatch.link_batch(ei, ids, P,
                                  generator=torch.Generator(device=DEV).manual_seed(100 + b))
        lb.mb = s.sample(lb.seeds, seed=b)
        step.prepare(lb.mb, lb.pu, lb.pp, lb.pn)
        want_b, want_l = barena.clone(), larena.clone()
        barena.fill_(0x5A)
        larena.fill_(0x5A)
        ls.prepare(ids, b, torch.Generator(device=DEV).manual_seed(100 + b))
        torch.cuda.synchronize()
        for name, (o, n, dt, nb) in step.blocks.arena.layout.items():
            assert torch.equal(barena[o:o + nb], want_b[o:o + nb]), (b, name)
        for name, (o, n, dt, nb) in ll.arena.layout.items():
            assert torch.equal(larena[o:o + nb], want_l[o:o + nb]), (b, name)
        assert int(ls.edge_count()) == sum(c.num_edges for blk in lb.mb.blocks
                                           for c in blk.csr.values())
    # one captured step over LinkSampler-staged batches
    lb0 = minibatch.link_batch(ei, order[:B], P)
    lb0.mb = s.sample(lb0.seeds, seed=0)
    ll.load(lb0.pu, lb0.pp, lb0.pn)
    step.capture(lb0.mb)
    ids = order[5 * B:6 * B]
    ls.prepare(ids, 5, torch.Generator(device=DEV).manual_seed(9))
    got = float(step.step())
    lb = minibatch.link_batch(ei, ids, P, generator=torch.Generator(device=DEV).manual_seed(9))
    lb.mb = s.sample(lb.seeds, seed=5)
    ref = _ref_link_loss(sampler.forward_blocks(model, lb.mb, g.x_dict), lb)
    assert abs(got - float(ref)) <= 2e-6 * abs(float(ref)), (got, float(ref))


@pytest.mark.parametrize("E,nu,np_", [(48, 48, 96), (1024, 1024, 2048), (1024, 2048, 3072),
                                      (3000, 2500, 6100)])
def test_link_group_equals_torch_grouping(E, nu, np_):
    """hgnn_link_group (LinkLoss.prepare's one call) against the torch grouping it replaced:
    pairs by user (stable), their posts / negatives / users in that order, the same pairs by
    post (stable transpose: users and CSR positions), the negatives by post (users in order) —
    at the bench's batch size too (B = 1024 pairs over 1024 users / 2048 posts)."""
    from truth_recommendation_gnn_amd import _native as N
    gen = torch.Generator(device=DEV).manual_seed(E)
    pu = torch.randint(0, nu, (E,), device=DEV, generator=gen, dtype=torch.int32)
    pp = torch.randint(0, np_, (E,), device=DEV, generator=gen, dtype=torch.int32)
    pn = torch.randint(0, np_, (E,), device=DEV, generator=gen, dtype=torch.int32)
    i32 = dict(dtype=torch.int32, device=DEV)
    out = {k: torch.full((n,), -7, **i32) for k, n in (
        ("rowptr", nu + 1), ("col", E), ("neg", E), ("uop", E), ("p_rowptr", np_ + 1),
        ("p_users", E), ("p_perm", E), ("n_rowptr", np_ + 1), ("n_users", E))}
    ws = torch.empty(int(N.lib().hgnn_link_group_ws_bytes(E)), dtype=torch.uint8, device=DEV)
    N.check(N.lib().hgnn_link_group(
        N.ptr(pu), N.ptr(pp), N.ptr(pn), E, nu, np_,
        *[N.ptr(out[k]) for k in ("rowptr", "col", "neg", "uop", "p_rowptr", "p_users",
                                  "p_perm", "n_rowptr", "n_users")],
        N.ptr(ws), ws.numel(), N.stream_ptr(DEV)), "hgnn_link_group")
    order = torch.argsort(pu.long(), stable=True)
    rowptr = torch.zeros(nu + 1, dtype=torch.long, device=DEV)
    rowptr[1:] = torch.cumsum(torch.bincount(pu.long(), minlength=nu), 0)
    col, neg, uop = pp[order], pn[order], pu[order]
    assert torch.equal(out["rowptr"].long(), rowptr)
    assert torch.equal(out["col"], col) and torch.equal(out["neg"], neg)
    assert torch.equal(out["uop"], uop)
    po = torch.argsort(col.long(), stable=True)            # positions by post, stable
    prow = torch.zeros(np_ + 1, dtype=torch.long, device=DEV)
    prow[1:] = torch.cumsum(torch.bincount(col.long(), minlength=np_), 0)
    assert torch.equal(out["p_rowptr"].long(), prow)
    assert torch.equal(out["p_perm"].long(), po) and torch.equal(out["p_users"], uop[po])
    no = torch.argsort(neg.long(), stable=True)
    nrow = torch.zeros(np_ + 1, dtype=torch.long, device=DEV)
    nrow[1:] = torch.cumsum(torch.bincount(neg.long(), minlength=np_), 0)
    assert torch.equal(out["n_rowptr"].long(), nrow) and torch.equal(out["n_users"], uop[no])
