#!/usr/bin/env python3
"""The cfg5 replay's kernels per step from a kernel-trace tail (scripts/gpu_r6_cfg5_trace.sh):
splits the trace at each fused-Adam kernel (the last node of a step), and for the last full
step prints every kernel of the replay's queue with its duration and the gap before it, plus
the other queue's (the sampler's) kernels in the same window.

  python scripts/cfg5_trace_nodes.py gpurun_out/r6_cfg5_trace_tail.csv"""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["start"], r["dur"] = int(r["start_ns"]), int(r["dur_ns"])
    adam = [i for i, r in enumerate(rows) if "adam" in r["name"].lower()]
    if len(adam) < 2:
        raise SystemExit("fewer than two Adam kernels in the tail")
    a0, a1 = adam[-2], adam[-1]
    q = rows[a1]["queue"]
    step = [r for r in rows[a0 + 1:a1 + 1]]
    main_q = [r for r in step if r["queue"] == q]
    other = [r for r in step if r["queue"] != q]
    t0 = rows[a0]["start"] + rows[a0]["dur"]
    t1 = rows[a1]["start"] + rows[a1]["dur"]
    print(f"step window {(t1 - t0) / 1e3:.1f} us; replay queue {q}: {len(main_q)} kernels, "
          f"busy {sum(r['dur'] for r in main_q) / 1e3:.1f} us; other queues: {len(other)} kernels, "
          f"busy {sum(r['dur'] for r in other) / 1e3:.1f} us")
    prev = t0
    for r in main_q:
        print(f"  gap {(r['start'] - prev) / 1e3:6.1f}  dur {r['dur'] / 1e3:6.1f}  grid {r['grid']:>9}  "
              f"{r['name'][:100]}")
        prev = r["start"] + r["dur"]
    c = collections.Counter(r["name"].split("(")[0][:60] for r in other)
    print("other queues:", dict(c))


if __name__ == "__main__":
    main(sys.argv[1])
