"""GPU, world_size 2 on one device (gloo over device tensors): parallel.UserShard on the HIP
kernels, with the forward all-reduces in flight during the user-side layer and the backward one
handed on unfinished to its consumer (ops.await_pending), reproduces the golden single-process
step: loss and every parameter gradient.  (RCCL needs one GPU per rank; the collective logic is
the same, and the 8-GPU runs are the driver's.)"""
import os
import pathlib
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

GOLD = pathlib.Path(__file__).resolve().parent / "golden"
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from truth_recommendation_gnn_amd import HeteroSAGE, parallel
        dev = torch.device("cuda:0")
        z = np.load(GOLD / "cfg2_slice_hetero_sage.npz")
        ei = torch.from_numpy(z["ei_engages"]).to(dev)
        xu = torch.from_numpy(z["x_user"]).to(dev)
        xp = torch.from_numpy(z["x_post"]).to(dev)
        params = {k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param:")}
        model = HeteroSAGE(64, parallel.RELATIONS, num_layers=2).to(dev)
        model.load_state_dict(params)
        pw = torch.from_numpy(z["pos_weights"]).to(dev)
        env = parallel.DistEnv.from_torch()
        shard = parallel.UserShard(ei, xu.shape[0], xp.shape[0], env, pos_weights=pw)
        assert shard.impl.defer_grad
        h_u, h_p = shard.forward(model, xu[shard.lo:shard.hi].contiguous(), xp)
        neg = shard.local_edges_of(torch.from_numpy(z["neg_p"]).to(dev))
        loss = shard.loss(h_u, h_p, neg)
        loss.backward()
        parallel.sync_grads(model, env)
        total = env.all_reduce_(loss.detach().clone())
        torch.cuda.synchronize()
        if rank == 0:
            q.put((float(total), {n: p.grad.cpu().numpy() for n, p in model.named_parameters()},
                   h_p.detach()[:xp.shape[0]].cpu().numpy()))
    except Exception as e:   # surface worker failures in the parent
        q.put(repr(e))
        raise
    finally:
        dist.destroy_process_group()


def test_user_shard_world2_async_collectives_match_golden():
    z = np.load(GOLD / "cfg2_slice_hetero_sage.npz")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert not isinstance(res, str), res
    loss, grads, h_p = res
    assert abs(loss - float(z["loss"])) <= 1e-4 * abs(float(z["loss"]))
    np.testing.assert_allclose(h_p, z["out_post"], rtol=1e-4, atol=1e-5 * np.abs(z["out_post"]).max())
    for name, g in grads.items():
        ref = z["grad:" + name]
        np.testing.assert_allclose(g, ref, rtol=1e-4, atol=1e-5 * max(np.abs(ref).max(), 1e-6))
