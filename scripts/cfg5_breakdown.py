"""Where a cfg5 mini-batch step's time goes: per phase (sample, forward, loss, backward, Adam) the
host issue time (perf_counter up to the last launch) and the wall time to completion (after a
device sync), over 30 steps after 5 warm-ups.  Phases are synchronised here, so the total is
above bench.py's pipelined ms/step; the host column is what bounds the step when the GPU idles.
usage: python scripts/cfg5_breakdown.py [--scale S]"""
import argparse
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from truth_recommendation_gnn_amd import HeteroSAGE, sampler, synth  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--cprofile", action="store_true", help="also cProfile the recorded steps")
    a = ap.parse_args()
    dev = torch.device("cuda")
    cfg = synth.CONFIGS["cfg5"] if a.scale == 1.0 else synth.scaled("cfg5", a.scale)
    g = synth.make_graph(cfg, device=dev, device_gen=True)
    rels = bench.relations_of(cfg)
    s = sampler.NeighborSampler({"user": cfg.num_users, "post": cfg.num_posts},
                                g.edge_index_dict, [et for et, _ in rels], [15, 10])
    torch.manual_seed(synth.WEIGHT_SEED)
    model = HeteroSAGE(cfg.hidden, rels, num_layers=cfg.layers, in_channels=cfg.dim).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    gen = torch.Generator(device=dev).manual_seed(0)
    order = {"user": torch.randperm(cfg.num_users, device=dev, generator=gen),
             "post": torch.randperm(cfg.num_posts, device=dev, generator=gen)}
    phases = ["sample", "forward", "loss", "backward", "adam"]
    host = {p: [] for p in phases}
    wall = {p: [] for p in phases}

    def step(i, record):
        seeds = {t: o[i * 1024:(i + 1) * 1024] for t, o in order.items()}
        marks = []
        t0 = time.perf_counter()
        mb = s.sample(seeds, seed=i)
        marks.append(("sample", t0, time.perf_counter()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = sampler.forward_blocks(model, mb, g.x_dict)
        marks.append(("forward", t0, time.perf_counter()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        u, p = out["user"], out["post"]
        pos = (u * p).sum(1)
        neg = (u * p.roll(1, 0)).sum(1)
        loss = (torch.nn.functional.softplus(-pos).mean()
                + torch.nn.functional.softplus(neg).mean())
        marks.append(("loss", t0, time.perf_counter()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        marks.append(("backward", t0, time.perf_counter()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opt.step()
        marks.append(("adam", t0, time.perf_counter()))
        torch.cuda.synchronize()
        t_end = time.perf_counter()
        if record:
            ends = [m[1] for m in marks[1:]] + [t_end]
            for (name, t_a, t_b), t_c in zip(marks, ends):
                host[name].append((t_b - t_a) * 1e3)
                wall[name].append((t_c - t_a) * 1e3)

    for i in range(5):
        step(i, False)
    prof = None
    if a.cprofile:
        import cProfile
        # backward on this thread, so cProfile sees the autograd functions' Python
        torch.autograd.set_multithreading_enabled(False)
        prof = cProfile.Profile()
        prof.enable()
    for i in range(5, 5 + a.steps):
        step(i, True)
    if prof is not None:
        import pstats
        prof.disable()
        st = pstats.Stats(prof)
        st.sort_stats("tottime").print_stats(40)
        st.sort_stats("cumtime").print_stats(80)
    print(f"{'phase':10s} {'host ms':>8s} {'wall ms':>8s}")
    for p in phases:
        print(f"{p:10s} {statistics.median(host[p]):8.3f} {statistics.median(wall[p]):8.3f}")
    print(f"{'total':10s} {sum(statistics.median(host[p]) for p in phases):8.3f} "
          f"{sum(statistics.median(wall[p]) for p in phases):8.3f}")


if __name__ == "__main__":
    main()
