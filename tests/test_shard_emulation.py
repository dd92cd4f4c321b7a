"""CPU: scripts/shard_emulation.py's stand-in environment (every collective replaced by a local
copy of the same shape) still drives the real ``UserShard.step`` end to end — it must accept
every call the sharded step makes (round 4 added ``reduce_scatter_async(..., out=)``, which the
stand-in lacked until a GPU run failed on it).  The numbers are not checked (the stand-ins sum
nothing); the step's completion and a finite loss and gradient for every parameter are."""
import importlib.util
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _emulation_module():
    spec = importlib.util.spec_from_file_location(
        "shard_emulation", os.path.join(ROOT, "scripts", "shard_emulation.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("kind,world,slice_inputs", [("engage2", 2, True), ("engage2", 3, False),
                                                     ("tiny_rgcn", 2, False)])
def test_emulated_step_runs_the_sharded_schedule(kind, world, slice_inputs):
    from dist_cases import setup
    from dist_torch_impl import TorchImpl
    from truth_recommendation_gnn_amd import synth
    from truth_recommendation_gnn_amd.parallel import UserShard, user_range
    emu = _emulation_module()
    torch.manual_seed(0)
    cfg, g, model, params, _, edges = setup(kind)
    model.load_state_dict(params)
    pos = g.edge_index_dict[synth.ENGAGES]
    neg = synth.negative_posts(cfg.num_posts, pos.shape[1])
    pw = synth.interaction_weights(cfg.num_posts)[pos[1]]
    for rank in range(world):
        env = emu.EmulEnv(world=world, rank=rank)
        shard = UserShard(edges, cfg.num_users, cfg.num_posts, env, impl=TorchImpl(),
                          pos_weights=pw, slice_inputs=slice_inputs)
        lo, hi = user_range(cfg.num_users, world, rank)
        for p in model.parameters():
            p.grad = None
        loss = shard.step(model, g.x_dict["user"][lo:hi], g.x_dict["post"],
                          shard.local_edges_of(neg),
                          x_user_full=g.x_dict["user"] if slice_inputs else None)
        assert torch.isfinite(loss).all()
        for n, p in model.named_parameters():
            assert p.grad is not None and torch.isfinite(p.grad).all(), n
