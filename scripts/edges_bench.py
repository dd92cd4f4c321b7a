"""Edge construction from raw ids: device path vs the reference's host loop.

Workload: a cfg2-sized activity frame — E rows of (engager, target_user: string user ids out of U,
post_id: int out of P), ~2% of ids unmapped — mapped by ``edges.build_edge_index_safe``
(train_gnn.py:40-73).  Reported:
  * device time of lookups + compaction (HIP events; inputs already encoded and resident),
  * end-to-end time from the pandas frame (includes the Arrow conversion of the string columns,
    the host->device copies and the single size sync),
  * the reference loop (oracle/edges_ref.py, iterrows + dict.get) on a bounded sample, as rows/s.
Run on the GPU box:  python scripts/edges_bench.py [--rows 20000000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from truth_recommendation_gnn_amd import edges  # noqa: E402
from oracle import edges_ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20_000_000)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--posts", type=int, default=100_000)
    ap.add_argument("--sample", type=int, default=100_000)
    a = ap.parse_args()
    dev = torch.device("cuda")
    rng = np.random.default_rng(0)
    users = np.array([f"{rng.integers(10**17, 10**18)}" for _ in range(a.users)], dtype=object)
    user_to_idx = {u: i for i, u in enumerate(sorted(set(users)))}
    post_to_idx = {i: len(user_to_idx) + i for i in range(a.posts)}
    pool = np.concatenate([users, np.array(["unknown_a", "unknown_b"], dtype=object)])

    def col():
        j = rng.integers(0, a.users, a.rows)
        j[rng.random(a.rows) < 0.01] = a.users          # ~1% unmapped per user column
        return pool[j]

    posts = rng.integers(0, a.posts + a.posts // 100, a.rows)   # ~1% out of range
    df = pd.DataFrame({"engager": col(), "target_user": col(), "post_id": posts})
    print(f"frame ready: {a.rows} rows", flush=True)

    t0 = time.perf_counter()
    um, pm = edges.IdMap(user_to_idx, dev), edges.IdMap(post_to_idx, dev)
    torch.cuda.synchronize()
    t_maps = time.perf_counter() - t0

    # end to end from the frame (warm once, then time)
    edges.build_edge_index_safe(df.iloc[:1000], um, pm, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng, auth = edges.build_edge_index_safe(df, um, pm, device=dev)
    torch.cuda.synchronize()
    t_e2e = time.perf_counter() - t0

    # the same frame with Arrow-backed string columns (no per-row host conversion)
    dfa = df.astype({"engager": "string[pyarrow]", "target_user": "string[pyarrow]"})
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    edges.build_edge_index_safe(dfa, um, pm, device=dev)
    torch.cuda.synchronize()
    t_e2e_arrow = time.perf_counter() - t0
    del dfa

    # device part only: queries pre-encoded and resident
    qe, qt, qp = (edges._encode(df[c]) for c in ("engager", "target_user", "post_id"))

    # resident-input timing: encode to device tensors once, time the kernels with events
    lib = edges.N.lib()
    st = torch.cuda.current_stream()
    dq = {}
    for name, q in (("engager", qe), ("target_user", qt)):
        offs, data, valid = q.strs
        dq[name] = (edges._h2d(offs, dev), edges.bytes_to_device(data, dev),
                    edges._h2d(valid, dev))
    pq = torch.from_numpy(qp.ints[0]).to(dev)
    outs = {k: torch.empty(a.rows, dtype=torch.int64, device=dev)
            for k in ("engager", "target_user", "post_id")}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for it in range(3):
        ev[0].record(st)
        for name in ("engager", "target_user"):
            o, d, v = dq[name]
            um._lookup(um._str, None, o, d, v, a.rows, outs[name])
        pm._lookup(pm._int, pq, None, None, None, a.rows, outs["post_id"])
        ev[1].record(st)
        edges.compact_rows([outs["engager"], outs["post_id"], outs["target_user"]],
                           [(0, 1), (1, 2)])
        ev[2].record(st)
        torch.cuda.synchronize()
    t_lookup = ev[0].elapsed_time(ev[1]) * 1e-3
    t_compact = ev[1].elapsed_time(ev[2]) * 1e-3

    # reference loop on a bounded sample
    s = df.iloc[: a.sample]
    t0 = time.perf_counter()
    ref_e, ref_a = edges_ref.build_edge_index_safe(s, user_to_idx, post_to_idx)
    t_ref = time.perf_counter() - t0
    got_e, got_a = edges.build_edge_index_safe(s, um, pm, device=dev)
    assert torch.equal(got_e.cpu(), ref_e) and torch.equal(got_a.cpu(), ref_a)

    str_bytes = sum(int(dq[k][1].numel()) for k in dq)
    # algorithmic bytes of the lookups: per query its offsets (16 B) + bytes + valid (1 B), one
    # 16-B slot probe + the matched key's offsets (16 B) and bytes + the value (8 B) + out (8 B)
    res = {
        "rows": a.rows, "kept": int(eng.shape[1]),
        "build_maps_s": round(t_maps, 3),
        "end_to_end_s": round(t_e2e, 3), "end_to_end_rows_per_s": a.rows / t_e2e,
        "end_to_end_arrow_columns_s": round(t_e2e_arrow, 3),
        "device_lookup_ms": round(t_lookup * 1e3, 3), "device_compact_ms": round(t_compact * 1e3, 3),
        "device_rows_per_s": a.rows / (t_lookup + t_compact),
        "query_string_bytes": str_bytes,
        "reference_loop_rows_per_s": a.sample / t_ref, "reference_sample_rows": a.sample,
        "speedup_end_to_end_vs_reference": (a.rows / t_e2e) / (a.sample / t_ref),
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
