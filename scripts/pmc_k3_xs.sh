#!/bin/bash
# Where the split-once K3 kernels' cycles go at the cfg4 9M-row shapes (scripts/k3_xs_target.py):
# MFMA busy, wave-cycle breakdown, instruction mix, LDS conflicts.  Separate --pmc passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4}
i=0
for c in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
         "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
         "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmcxs_${TAG}_$i -o k -- python3 scripts/k3_xs_target.py > gpurun_out/pmcxs_${TAG}_$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 gpurun_out/pmcxs_${TAG}_$i.log; exit 1; }
done
export TAG
python3 - <<'PY' > gpurun_out/pmc_k3_cfg4_${TAG}.json && cat gpurun_out/pmc_k3_cfg4_${TAG}.json
import collections, csv, glob, json, os
tag = os.environ["TAG"]
out = {"note": "cfg4 9M-row K3 launches (scripts/k3_xs_target.py, 3 of each); per-launch means; "
               "GRBM_GUI_ACTIVE is summed over the 8 XCDs, mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / "
               "(1024 SIMDs x GRBM_GUI_ACTIVE / 8); SQ_WAVE_CYCLES / SQ_WAIT_* in quad-cycles",
       "kernels": {}}
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/pmcxs_{tag}_[0-9]/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "hgnn" in r["Kernel_Name"]:
            acc[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
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
PY
