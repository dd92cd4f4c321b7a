"""Experiment: the loss's dP gather (hgnn_score_gather2: positives + negatives grouped by post,
U rows from the 4.6 GB user table) at cfg4 as one pass vs B passes over user blocks (positives
and negatives of block b per pass, accumulating into dP).  Prints ms per full dP gather.
usage: python scripts/score_block_bench.py [B ...]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from truth_recommendation_gnn_amd import _native as N, graph, ops, synth  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda")
    cfg = synth.CONFIGS["cfg4"]
    t0 = time.time()
    g = synth.make_graph(cfg, device=dev, device_gen=True)
    pos = g.edge_index_dict[synth.ENGAGES]            # user -> post
    n_u, n_p, d = cfg.num_users, cfg.num_posts, cfg.hidden
    del g
    U = torch.randn(n_u, d, device=dev) * 0.1
    P = torch.randn(n_p, d, device=dev) * 0.1
    neg = torch.stack([pos[0], torch.randint(0, n_p, (pos.shape[1],), device=dev)])
    print(f"setup {time.time() - t0:.1f}s", flush=True)
    pc = graph.relation_csr(pos, n_u, n_p)
    nc = graph.RelationCSR(neg, n_u, n_p, chunk=graph.NO_SPLIT)
    c = torch.tensor(1.3, device=dev)
    inv_e = 1.0 / pos.shape[1]
    ref = torch.empty(n_p, d, device=dev)
    t_one = timed(lambda: ops._score_gather2(U, P, pc.fwd, nc.fwd, c, inv_e, ref))
    print(f"B=1 {t_one:.3f} ms", flush=True)
    for B in [int(b) for b in sys.argv[1:]] or [4, 8]:
        pp, _ = pc.blocks("fwd", B)
        npass, _ = nc.blocks("fwd", B)
        out = torch.empty_like(ref)
        lib = N.lib()

        def run():
            s = N.stream_ptr(dev)
            for b in range(B):
                gp, gn = pp[b], npass[b]
                p = gp.plan
                slab = (torch.empty(p.n_chunks * d, device=dev) if p.n_heavy else None)
                if b == 0:
                    N.check(lib.hgnn_score_gather2(
                        N.ptr(U), n_u, N.ptr(P), d, N.ptr(gp.rowptr), N.ptr(gp.col),
                        N.ptr(gn.rowptr), N.ptr(gn.col), n_p, N.ptr(c), inv_e,
                        N.ptr(p.heavy_rows), N.ptr(p.heavy_first), p.n_heavy, p.n_chunks,
                        p.chunk, N.ptr(slab), N.ptr(out), s), "sg2")
                else:   # accumulate: positives then negatives as two score gathers
                    for grp, mode in ((gp, 1), (gn, 2)):
                        q = grp.plan
                        sl = (torch.empty(q.n_chunks * d, device=dev) if q.n_heavy else None)
                        N.check(lib.hgnn_score_gather(
                            N.ptr(U), n_u, N.ptr(P), d, N.ptr(grp.rowptr), N.ptr(grp.col), n_p,
                            mode, N.ptr(c), inv_e, N.ptr(q.heavy_rows), N.ptr(q.heavy_first),
                            q.n_heavy, q.n_chunks, q.chunk, N.ptr(sl), N.ptr(out), 1, s), "sg")
        t = timed(run)
        err = float((out - ref).abs().max() / ref.abs().max())
        print(f"B={B} {t:.3f} ms ({t_one / t:.3f}x) rel_err={err:.2e}", flush=True)


if __name__ == "__main__":
    main()
