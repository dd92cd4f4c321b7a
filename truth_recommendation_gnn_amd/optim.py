"""Adam for the rebuilt training step: ``torch.optim.Adam``'s update (the reference's optimizer,
``train_gnn.py:207``: ``Adam(model.parameters(), lr=0.001)``) as ONE native launch over every
parameter (``hgnn_adam_multi``, ``csrc/adam.hip``).

Capturable by construction: the step count of each parameter group is a device float that the
launch itself advances, so a recorded step (``minibatch.CapturedStep``) replays the update with
no host value and one graph node (torch's capturable fused Adam: a step-tensor add plus the
update, two nodes).  The arithmetic follows torch's fused kernel (fp32 state, double
hyper-parameters); ``tests/test_gpu_parity.py::test_adam_matches_torch`` holds it to torch's
``Adam(fused=True)``.  GPU only: a CPU parameter raises (the product path has no fallback).
"""
from typing import Iterable

import torch

from . import _native as N


class Adam(torch.optim.Optimizer):
    """``torch.optim.Adam`` (no amsgrad / maximize; L2 ``weight_decay`` as torch's original mode)
    over fp32 CUDA parameters."""

    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError(f"Adam: invalid hyper-parameters lr={lr} betas={betas} eps={eps} "
                             f"weight_decay={weight_decay}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay))

    def _group_state(self, group, dev):
        """The group's device step count and the launch's block counter (zeroed once, eagerly:
        the first step runs before any capture)."""
        st = group.get("_dev_state")
        if st is None:
            st = (torch.zeros(1, dtype=torch.float32, device=dev),
                  torch.zeros(1, dtype=torch.int32, device=dev))
            group["_dev_state"] = st
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            dev = ps[0].device
            for p in ps:
                if p.device.type != "cuda" or p.dtype != torch.float32 or p.grad.is_sparse:
                    raise RuntimeError("optim.Adam: fp32 dense CUDA parameters only "
                                       f"(got {p.dtype} on {p.device})")
                if not (p.is_contiguous() and p.grad.is_contiguous()):
                    raise RuntimeError("optim.Adam: contiguous parameters and gradients only")
            ms, vs = [], []
            for p in ps:
                s = self.state[p]
                if not s:
                    s["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    s["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                ms.append(s["exp_avg"])
                vs.append(s["exp_avg_sq"])
            step_t, done = self._group_state(group, dev)
            b1, b2 = group["betas"]
            N.check(N.lib().hgnn_adam_multi(
                len(ps), N.ptr_array(ps), N.ptr_array([p.grad for p in ps]), N.ptr_array(ms),
                N.ptr_array(vs), N.i64_array([p.numel() for p in ps]), N.ptr(step_t), N.ptr(done),
                float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                float(group["weight_decay"]), N.stream_ptr(dev)), "hgnn_adam_multi")
        return loss

    def steps_done(self, group: int = 0) -> int:
        """The group's step count (a host read: not inside a capture)."""
        st = self.param_groups[group].get("_dev_state")
        return 0 if st is None else int(st[0].item())
