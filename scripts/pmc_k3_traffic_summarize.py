#!/usr/bin/env python3
"""HBM traffic of the four 9M-row K3 launches of the cfg4 step (scripts/k3_xs_target.py under
separate FETCH_SIZE / WRITE_SIZE passes, scripts/pmc_k3_traffic.sh) against the algorithmic bytes
the bench's per-kernel timer counts for the same launches (the target's K3_ALG line).  gfx950
correction as scripts/pmc_step_summarize.py: read bytes = 2 x FETCH_SIZE.  Writes the
`launches` entries bench.py looks up (cfg4|n1|linear_*) and, with --merge FILE, adds them to that
PMC summary.  usage: pmc_k3_traffic_summarize.py <fetch_dir> <write_dir> <target_log> [--merge F]"""
import collections
import csv
import glob
import json
import sys

# template -> the bench label of its 9M-row launch in the cfg4 step
ROLE = {"k_lin_fwd_xs<256, false>": "linear_fwd[{n}x256->128]",
        "k_lin_bwd_xs<256, false, true, false>": "linear_bwd[{n}x256->128]",
        "k_lin_fwd_xs<128, true>": "linear_fwd[{n}x128->128]",
        "k_lin_bwd_xs<128, true, true, false>": "linear_bwd[{n}x128->128]"}


def per_kernel(d, counter):
    out = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                out[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    fetch_dir, write_dir, log = sys.argv[1:4]
    alg = None
    for line in open(log):
        if line.startswith("K3_ALG "):
            alg = json.loads(line[len("K3_ALG "):])
    n = alg["n"]
    fetch, write = per_kernel(fetch_dir, "FETCH_SIZE"), per_kernel(write_dir, "WRITE_SIZE")
    launches = {}
    for frag, lab in ROLE.items():
        lab = lab.format(n=n)
        fv = [v for k, vs in fetch.items() if frag in k for v in vs]
        wv = [v for k, vs in write.items() if frag in k for v in vs]
        if not fv or not wv:
            continue
        hbm = (2 * sum(fv) / len(fv) + sum(wv) / len(wv)) * 1024
        ab = alg["bytes"].get(lab)
        launches[f"cfg4|n1|{lab}"] = {
            "kernels": [frag], "dispatches": len(fv), "hbm_bytes_per_launch": int(hbm),
            "alg_bytes_per_launch": int(ab) if ab else None,
            "traffic_over_algorithmic": round(hbm / ab, 3) if ab else None,
            "source": "scripts/k3_xs_target.py (the step's four 9M-row K3 launches, 4 of each)"}
    out = {"launches": launches}
    if "--merge" in sys.argv:
        path = sys.argv[sys.argv.index("--merge") + 1]
        pm = json.load(open(path))
        pm.setdefault("launches", {}).update(launches)
        pm.setdefault("kernels", {}).update({k.split("|")[-1]: v for k, v in launches.items()})
        open(path, "w").write(json.dumps(pm, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
