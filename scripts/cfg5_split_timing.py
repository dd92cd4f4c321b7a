#!/usr/bin/env python3
"""What bounds the cfg5 step: the sampler alone (link batch + 2-hop sample per batch, on one
stream, host-timed over N batches) against the captured step's replay alone (the same batch
loaded and replayed N times).  usage: python scripts/cfg5_split_timing.py [N]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from truth_recommendation_gnn_amd import minibatch, sampler  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
captured = {}
orig = minibatch.CapturedStep.capture


def keep(self, *a, **k):
    orig(self, *a, **k)
    captured["step"] = self


minibatch.CapturedStep.capture = keep
orig_sample = sampler.NeighborSampler.sample
samplers = {}


def keep_s(self, *a, **k):
    samplers["s"] = self
    return orig_sample(self, *a, **k)


sampler.NeighborSampler.sample = keep_s
bench.main(["--config", "cfg5", "--steps", "50", "--warmup", "10", "--no-cpu-baseline",
            "--timer-steps", "0"])
step, s = captured["step"], samplers["s"]
dev = torch.device("cuda")
seeds = {"user": torch.randint(0, 9_000_000, (1024,), device=dev).unique(),
         "post": torch.randint(0, 1_000_000, (2048,), device=dev).unique()}
mb = s.sample(seeds, seed=1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(N):
    s.sample(seeds, seed=i)
torch.cuda.synchronize()
t1 = time.perf_counter()
for i in range(N):
    step.step(mb)
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"sampler alone {(t1 - t0) / N * 1e3:.3f} ms/batch; replay alone {(t2 - t1) / N * 1e3:.3f} "
      f"ms/step (load + replay)")
