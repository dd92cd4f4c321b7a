"""CPU, gloo, world 8 (and 3): every rank of the sharded training step issues the SAME sequence of
collectives — op, shape, dtype — from the shard's construction through ``UserShard.step`` and the
gradient all-reduce, whatever its local sizes.  RCCL matches collectives by issue
order only: a rank that skips one, or issues another shape, hangs the whole job until the
process-group timeout, so this is checked before the first 8-GPU run rather than by it.

The graphs hold ranks with no users at all (tiny4 at world 8: 7 users), no engages edge, no halo
row, and (engage2 at world 8) every rank with edges.  ``all_to_all_single`` carries per-rank split
sizes by design (the halo), so only its row width and dtype must agree; its calls are still
counted and ordered with the rest."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

_OPS = ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor", "all_gather",
        "broadcast", "all_to_all_single", "barrier")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sig(name, args, kwargs):
    """What must agree across ranks for collective ``name``."""
    tensors = [a for a in args if isinstance(a, torch.Tensor)]
    if name == "all_gather":
        lst = args[0]
        return (name, len(lst), tuple(lst[0].shape), str(lst[0].dtype))
    if name == "barrier":
        return (name,)
    if name == "all_to_all_single":
        out, inp = tensors[0], tensors[1]
        return (name, tuple(out.shape[1:]), str(out.dtype))
    if name == "broadcast":
        return (name, tuple(tensors[0].shape), str(tensors[0].dtype),
                int(kwargs.get("src", args[1] if len(args) > 1 else -1)))
    return (name,) + tuple((tuple(t.shape), str(t.dtype)) for t in tensors)


def _worker(rank, world, port, q, kind, slice_inputs, steps):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from dist_cases import setup as _setup
    from dist_torch_impl import TorchImpl
    from truth_recommendation_gnn_amd import synth
    from truth_recommendation_gnn_amd.parallel import DistEnv, UserShard, sync_grads, user_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    log = []
    orig = {n: getattr(dist, n) for n in _OPS}

    def wrap(n):
        def f(*a, **k):
            log.append(_sig(n, a, k))
            return orig[n](*a, **k)
        return f
    try:
        torch.set_num_threads(1)
        for n in _OPS:
            setattr(dist, n, wrap(n))
        env = DistEnv.from_torch()
        cfg, g, model, params, _, edges = _setup(kind)
        pos = g.edge_index_dict[synth.ENGAGES]
        pw = synth.interaction_weights(cfg.num_posts)[pos[1]]
        model.load_state_dict(params)
        shard = UserShard(edges, cfg.num_users, cfg.num_posts, env, impl=TorchImpl(),
                          pos_weights=pw, slice_inputs=slice_inputs)
        n_setup = len(log)
        full = g.x_dict["user"] if slice_inputs else None
        lo, hi = user_range(cfg.num_users, world, rank)
        gen = torch.Generator().manual_seed(11 + rank)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        for _ in range(steps):           # bench.py's step: explicit schedule, all-reduce, Adam
            opt.zero_grad(set_to_none=True)
            neg = torch.randint(0, cfg.num_posts, (shard.pos_local.shape[1],), generator=gen)
            shard.step(model, g.x_dict["user"][lo:hi], g.x_dict["post"], neg,
                       neg_order="user", x_user_full=full)
            sync_grads(model, env)
            opt.step()
        for n in _OPS:
            setattr(dist, n, orig[n])
        q.put({"rank": rank, "log": log, "n_setup": n_setup, "users": hi - lo,
               "n_local": int(shard.pos_local.shape[1])})
    except Exception as e:   # report instead of leaving the parent waiting on the queue
        q.put({"rank": rank, "error": repr(e)})
        raise
    finally:
        for n in _OPS:
            setattr(dist, n, orig[n])
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,slice_inputs", [
    (8, "tiny4", True),      # 7 users on 8 ranks: rank 7 owns none; post->post and halo
    (8, "engage2", True),    # the bench's two-relation graph and slice_inputs, every rank busy
    (3, "tiny_rgcn", False),  # the reference WeightedRGCN; the last rank has no engages edge
])
def test_every_rank_issues_the_same_collective_sequence(world, kind, slice_inputs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kind, slice_inputs, 2))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
    errs = [r["error"] for r in res if "error" in r]
    assert not errs, errs
    ref = res[0]["log"]
    assert len(ref) > res[0]["n_setup"] > 0
    # the two steps issue the same collectives (no first-step-only exchange)
    per_step = (len(ref) - res[0]["n_setup"]) // 2
    assert ref[res[0]["n_setup"]:res[0]["n_setup"] + per_step] == ref[res[0]["n_setup"] + per_step:]
    for r in res[1:]:
        assert r["n_setup"] == res[0]["n_setup"], (r["rank"], r["n_setup"], res[0]["n_setup"])
        assert len(r["log"]) == len(ref), (r["rank"], len(r["log"]), len(ref))
        for i, (a, b) in enumerate(zip(r["log"], ref)):
            assert a == b, (r["rank"], i, a, b)
    if kind == "tiny4":
        assert any(r["users"] == 0 for r in res)          # a rank without users took part
    if kind == "tiny_rgcn":
        assert any(r["n_local"] == 0 for r in res)        # a rank without positive edges
