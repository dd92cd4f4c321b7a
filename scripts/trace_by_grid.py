#!/usr/bin/env python3
"""Per-(kernel, grid) summary of a rocprofv3 kernel trace.

rocprofv3's --stats groups launches by kernel symbol only, so the two K1 forward gathers of a step
(post<-user over 100k rows and user<-post over 1M rows, one template instantiation) share a line.
Grouping by grid size as well separates them, so the roofline kernel's average launch duration
can be compared with bench.py's HIP-event figure.

usage: python scripts/trace_by_grid.py <..._kernel_trace.csv> [out.csv]
"""
import collections
import csv
import sys


def main():
    src = sys.argv[1]
    rows = list(csv.DictReader(open(src)))
    if not rows:
        raise SystemExit("empty trace")
    cols = rows[0].keys()
    name_c = next(c for c in cols if c.lower() in ("kernel_name", "kernel-name", "name"))
    start_c = next(c for c in cols if "start" in c.lower())
    end_c = next(c for c in cols if "end" in c.lower())
    grid_c = [c for c in cols if c.lower().startswith("grid_size")]
    wg_c = [c for c in cols if c.lower().startswith("workgroup_size")]
    agg = collections.OrderedDict()
    for r in rows:
        key = (r[name_c], "x".join(r[c] for c in grid_c), "x".join(r[c] for c in wg_c))
        dur = int(r[end_c]) - int(r[start_c])
        a = agg.setdefault(key, [0, 0, None, 0])
        a[0] += 1
        a[1] += dur
        a[2] = dur if a[2] is None else min(a[2], dur)
        a[3] = max(a[3], dur)
    out = csv.writer(open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout)
    out.writerow(["Name", "Grid", "Workgroup", "Calls", "TotalNs", "AverageNs", "MinNs", "MaxNs"])
    for (name, grid, wg), (n, tot, lo, hi) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.writerow([name, grid, wg, n, tot, round(tot / n, 1), lo, hi])


if __name__ == "__main__":
    main()
