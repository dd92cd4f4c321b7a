#!/usr/bin/env python3
"""Per-rank compute of the sharded N-GPU bench step (``UserShard.step``), on one GPU.

Rank 0 of the weak-scaled graph (``synth.replicated(cfg, N)``: N x the users, posts and edges),
or with ``--strong`` of the config's own graph split N ways (BASELINE cfg4 on 8 GPUs), runs the
real sharded code path — its user range, the post-table slice, the explicit collective
schedule — with every collective replaced by a local stand-in of the same shape (reduce-scatter:
this rank's slice of its own partial sums; all-gather: the own slice tiled N times; all-reduce:
identity).  So it times what one rank computes at N GPUs, collectives excluded (RCCL needs one GPU
per rank); the numbers are wrong (local degrees, tiled tables), the work is not.
python scripts/shard_emulation.py --world 8 [--steps 20] [--config cfg4 --strong]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import HeteroSAGE, ops, parallel, synth  # noqa: E402

RELATIONS = [(synth.REV_ENGAGES, 1.0), (synth.ENGAGES, 1.0)]


XGMI_LINK_GBS = 153.0        # one xGMI link per direction (a ring step is bound by one link)
XGMI_LINKS = 7               # peer links per GPU (a direct all-to-all pattern uses all of them)


class _Issued:
    """A stand-in collective's handle: records, on the stream, when its consumer waits."""

    def __init__(self, log, rec):
        self.log, self.rec = log, rec

    def wait(self):
        if self.rec is not None and "wait" not in self.rec:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.rec["wait"] = ev
        return True


class EmulEnv(parallel.DistEnv):
    """``world`` ranks seen from ``rank``, every collective a local stand-in (timing only).
    With ``log`` (a list) each collective records an event on the main stream when it is issued
    (after its stand-in copy) and one when its consumer waits for it: the time between the two
    is the compute the real collective runs under."""
    log = None

    def use_side_adjoint(self, t):
        return False

    def all_reduce_(self, t):
        return t

    def _issued(self, name, recv_bytes):
        if self.log is None:
            return parallel._Done()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        rec = {"op": name, "recv_bytes": int(recv_bytes), "issue": ev}
        self.log.append(rec)
        return _Issued(self.log, rec)

    def reduce_scatter_async(self, full, out=None):
        S = full.shape[0] // self.world
        mine = full[self.rank * S:(self.rank + 1) * S]
        out = mine.clone() if out is None else out.copy_(mine)
        nbytes = full.numel() * full.element_size() * (self.world - 1) // self.world
        return out, self._issued("reduce_scatter", nbytes)

    def all_gather_async(self, own):
        out = own.repeat(self.world, *([1] * (own.dim() - 1)))
        return out, self._issued("all_gather", own.numel() * own.element_size() * (self.world - 1))

    def broadcast_slices_async(self, own):
        out = own.repeat(self.world, *([1] * (own.dim() - 1)))
        nb = own.numel() * own.element_size()
        return out, [parallel._Done() if q == self.rank else self._issued(f"broadcast[{q}]", nb)
                     for q in range(self.world)]

    def all_to_all_async(self, inp, send_splits, recv_splits):
        out = inp.new_zeros((int(sum(recv_splits)),) + tuple(inp.shape[1:]))
        return out, self._issued("all_to_all", out.numel() * out.element_size())

    def all_reduce_async(self, t):
        return self._issued("all_reduce", 2 * t.numel() * t.element_size() * (self.world - 1)
                            // self.world)


def link_timeline(log, t0, step_ms, gbs):
    """The recorded step replayed against one serial link of ``gbs`` GB/s: the collectives run
    in issue order, one at a time (one communicator), each recv_bytes / rate long, starting when
    issued and the link is free; a consumer that waits before its collective has ended stalls
    the compute (and every later issue) by the difference.  Returns the stall in total and per
    collective: the step at that link rate is the compute plus the stall."""
    ev = []
    for i, r in enumerate(log):
        ev.append((t0.elapsed_time(r["issue"]), 0, i))
        ev.append((t0.elapsed_time(r["wait"]) if "wait" in r else step_ms, 1, i))
    ev.sort()
    shift, free, end, stall = 0.0, 0.0, {}, [0.0] * len(log)
    for t, kind, i in ev:
        if kind == 0:
            start = max(t + shift, free)
            end[i] = free = start + log[i]["recv_bytes"] / (gbs * 1e9) * 1e3
        elif end[i] > t + shift:
            stall[i] = end[i] - (t + shift)
            shift += stall[i]
    return {"link_GBs": gbs, "step_ms_compute": round(step_ms, 3),
            "stall_ms": round(shift, 3), "step_ms_with_link": round(step_ms + shift, 3),
            "stall_ms_by_collective": [round(x, 3) for x in stall]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0, help="the rank whose share is emulated")
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--no-slice-inputs", action="store_true",
                    help="layer 1's post side through partial sums + reduce-scatter (round 1)")
    ap.add_argument("--strong", action="store_true",
                    help="partition the config's own graph (e.g. cfg4 over 8 ranks), not N x it")
    args = ap.parse_args()
    dev = torch.device("cuda")
    gcfg = synth.CONFIGS[args.config] if args.strong else synth.replicated(args.config, args.world)
    g = synth.make_graph(gcfg, device=dev, device_gen=True)
    pos_g = g.edge_index_dict[synth.ENGAGES]
    pw_g = synth.interaction_weights(gcfg.num_posts).to(dev)[pos_g[1]]
    env = EmulEnv(world=args.world, rank=args.rank)
    shard = parallel.UserShard({et: g.edge_index_dict[et] for et, _ in RELATIONS},
                               gcfg.num_users, gcfg.num_posts, env, pos_weights=pw_g,
                               slice_inputs=not args.no_slice_inputs)
    x_user = g.x_dict["user"][shard.lo:shard.hi].contiguous()
    x_full = None if args.no_slice_inputs else g.x_dict["user"]
    x_post = g.x_dict["post"]
    edges_local = sum(int(r.csr.num_edges) for r in shard.rels.values()) * gcfg.layers
    del g, pos_g, pw_g
    torch.cuda.empty_cache()
    model = HeteroSAGE(gcfg.hidden, RELATIONS, num_layers=gcfg.layers).to(dev)
    with torch.no_grad():
        shard.forward(model, x_user, x_post, x_user_full=x_full)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    gen = torch.Generator(device=dev).manual_seed(3)

    def step():
        if env.log is not None:                   # the step's start, for the link timeline
            env.t0 = torch.cuda.Event(enable_timing=True)
            env.t0.record()
        opt.zero_grad(set_to_none=True)
        neg = ops.draw_negatives(shard.pos_local, gcfg.num_posts, generator=gen)
        shard.step(model, x_user, x_post, neg, neg_order="user", x_user_full=x_full)
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    timer = ops.KernelTimer()                 # one more pass for the per-kernel split
    ops.set_timer(timer)
    for _ in range(args.steps):
        step()
    ops.set_timer(None)
    kern = {k: round(v["ms"] / args.steps, 4) for k, v in sorted(timer.summary().items())}
    # one more step with the collectives' issue / consumer-wait points recorded
    env.log = []
    step()
    flat = torch.cat([p.grad.reshape(-1) for p in model.parameters()])   # sync_grads' all-reduce
    env.all_reduce_async(flat).wait()
    t_end = torch.cuda.Event(enable_timing=True)
    t_end.record()
    torch.cuda.synchronize()
    step_ms = env.t0.elapsed_time(t_end)
    timeline = {f"{n}": link_timeline(env.log, env.t0, step_ms, XGMI_LINK_GBS * k)
                for n, k in (("1link_ring", 1), ("7links", XGMI_LINKS))}
    colls = []
    for r in env.log:
        cover = r["issue"].elapsed_time(r["wait"]) if "wait" in r else None
        t1 = r["recv_bytes"] / (XGMI_LINK_GBS * 1e9) * 1e3
        t7 = t1 / XGMI_LINKS
        colls.append({"op": r["op"], "recv_MB_per_rank": round(r["recv_bytes"] / 1e6, 1),
                      "issue_ms": round(env.t0.elapsed_time(r["issue"]), 3),
                      "wait_ms": round(env.t0.elapsed_time(r["wait"]), 3) if "wait" in r else None,
                      "cover_ms": None if cover is None else round(cover, 3),
                      "est_ms_1link_ring": round(t1, 3), "est_ms_7links": round(t7, 3),
                      "cover_over_1link": None if cover is None else round(cover / t1, 2) if t1 else None,
                      "cover_over_7links": None if cover is None else round(cover / t7, 2) if t7 else None})
    env.log = None
    print(json.dumps({"world": args.world, "rank": args.rank, "config": gcfg.name,
                      "chunk_group": parallel.CHUNK_GROUP, "chunk_first": parallel.CHUNK_FIRST,
                      "collectives": colls,
                      "link_timeline": timeline,
                      "scaling": "strong" if args.strong else "weak",
                      "users_own": shard.n_own, "posts_padded": shard.n_posts_pad,
                      "local_edges_per_step": edges_local,
                      "ms_per_step_compute": round(ms, 3),
                      "kernels_ms_per_step": kern, "kernels_sum_ms": round(sum(kern.values()), 3)}),
          flush=True)


if __name__ == "__main__":
    main()
