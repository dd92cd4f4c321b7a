#!/usr/bin/env python3
"""Per-kernel HBM traffic of the training step from separate rocprofv3 --pmc passes of
scripts/pmc_step_target.py (FETCH_SIZE; WRITE_SIZE), against each kernel's algorithmic bytes.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE tallies 128-B requests at 64 B, so read
bytes = 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B stores; both in KiB.  FETCH_SIZE counts
Infinity-Cache hits too (fabric requests leaving L2), so for tables under ~256 MiB "traffic" is
L2-miss traffic, not HBM bytes; at cfg4 the gathered user table is 4.6 GB.

usage: pmc_step_summarize.py <fetch_dir> <write_dir> <target_log> [out.json]"""
import collections
import csv
import glob
import json
import sys


def rows(d, counter, marker=None):
    """(kernel, grid) -> [values in dispatch order]; with ``marker``, only the dispatches after
    the last dispatch whose kernel name contains it (the profiled steps)."""
    out = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        recs = list(csv.DictReader(open(f)))
        key = "Dispatch_Id" if recs and "Dispatch_Id" in recs[0] else None
        if key:
            recs.sort(key=lambda r: int(r[key]))
        if marker and key:
            ids = [int(r[key]) for r in recs if marker in r["Kernel_Name"]]
            if ids:
                recs = [r for r in recs if int(r[key]) > max(ids)]
        for r in recs:
            if r["Counter_Name"] == counter:
                out[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return out


def match(kname, frag):
    frags = frag if isinstance(frag, list) else [frag]
    return any(f in kname for f in frags)


def main():
    fetch_dir, write_dir, log = sys.argv[1:4]
    info = None
    for line in open(log):
        if line.startswith("PMC_TARGET "):
            info = json.loads(line[len("PMC_TARGET "):])
    mk = info.get("marker")
    fetch, write = rows(fetch_dir, "FETCH_SIZE", mk), rows(write_dir, "WRITE_SIZE", mk)
    cfg, steps = info["config"], info["steps"]
    out = {"counters": "FETCH_SIZE, WRITE_SIZE (KiB): separate rocprofv3 --kernel-trace --pmc passes "
                       "of scripts/pmc_step_target.py",
           "correction": "hbm bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (gfx950 wide-read tally)",
           "config": cfg, "steps_profiled": steps, "launches": {}, "kernels": {}}
    for role, meta in info["roles"].items():
        grids = meta["grid"] if isinstance(meta["grid"], list) else [meta["grid"]]
        fk = [(k, v) for k, v in fetch.items() if match(k[0], meta["kernel"])
              and (meta["grid"] is None or k[1] in grids)]
        wk = [(k, v) for k, v in write.items() if match(k[0], meta["kernel"])
              and (meta["grid"] is None or k[1] in grids)]
        if not fk or not wk:
            continue
        f_tot = sum(sum(v) for _, v in fk)
        w_tot = sum(sum(v) for _, v in wk)
        n = sum(len(v) for _, v in fk)
        # launches of this role per profiled step (the sort is several kernels per call)
        calls = steps * meta["per_step"] if meta.get("per_step") else n
        hbm = (2 * f_tot + w_tot) * 1024 / calls
        rec = {"kernels": sorted({k[0].split("(")[0].replace("void ", "") for k, _ in fk}),
               "dispatches": n, "calls": calls, "fetch_kib_per_call": round(f_tot / calls, 1),
               "write_kib_per_call": round(w_tot / calls, 1), "hbm_bytes_per_launch": int(hbm),
               "alg_bytes_per_launch": meta["alg_bytes"],
               "traffic_over_algorithmic": (round(hbm / meta["alg_bytes"], 3)
                                            if meta["alg_bytes"] else None),
               "source": f"{cfg} step, {steps} steps"}
        out["kernels"][role] = rec
    # bench.py's kernel labels -> per-launch records (roofline.traffic lookup)
    U, P, d = info["U"], info["P"], info["d"]
    label = {"gather_fwd[post<-user]": f"gather_fwd[{P}<-{U}]x{d}",
             "gather_fwd[user<-post]": f"gather_fwd[{U}<-{P}]x{d}",
             "gather_bwd[post<-user]": f"gather_bwd[{P}<-{U}]x{d}",
             "gather_bwd[user<-post]": f"gather_bwd[{U}<-{P}]x{d}",
             "score_gather[post<-user]": f"score_gather[{P}<-{U}]x{d}",
             "edge_score": f"edge_score_d{d}", "sort_negatives": "sort_negatives"}
    for role, lab in label.items():
        if role in out["kernels"]:
            out["launches"][f"{cfg}|n1|{lab}"] = out["kernels"][role]
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(s + "\n")


if __name__ == "__main__":
    main()
