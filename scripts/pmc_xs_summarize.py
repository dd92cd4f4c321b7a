#!/usr/bin/env python3
"""Per-kernel means of the K3 PMC passes (scripts/pmc_k3_xs.sh): keyed by the kernel's name with
its template arguments, so each K3 variant gets its own row.

  python scripts/pmc_xs_summarize.py TAG > gpurun_out/pmc_k3_cfg4_TAG.json"""
import collections
import csv
import glob
import json
import re
import sys

tag = sys.argv[1]
out = {"note": "cfg4 9M-row K3 launches (scripts/k3_xs_target.py, 3 of each); per-launch means; "
               "GRBM_GUI_ACTIVE is summed over the 8 XCDs, mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / "
               "(1024 SIMDs x GRBM_GUI_ACTIVE / 8); SQ_WAVE_CYCLES / SQ_WAIT_* in quad-cycles",
       "kernels": {}}
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/pmcxs_{tag}_[0-9]/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "hgnn" not in r["Kernel_Name"]:
            continue
        m = re.search(r"(k_\w+(<[^()]*?>)?)\(", r["Kernel_Name"])
        acc[m.group(1) if m else r["Kernel_Name"][:80]][r["Counter_Name"]].append(
            float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    m = {c: sum(x) / len(x) for c, x in v.items()}
    if m.get("GRBM_GUI_ACTIVE"):
        m["mfma_util"] = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
    if m.get("SQ_INSTS_MFMA"):
        m["valu_per_mfma"] = m.get("SQ_INSTS_VALU", 0) / m["SQ_INSTS_MFMA"]
    if m.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in m:
                m[c + "_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
    out["kernels"][k] = {c: (round(x, 3) if abs(x) < 100 else round(x)) for c, x in m.items()}
print(json.dumps(out, indent=1))
