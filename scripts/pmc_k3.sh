#!/bin/bash
# PMC of the K3 kernels (scripts/k3_target.py): MFMA busy cycles vs GPU-active cycles, and the
# instruction mix.  Separate --pmc passes, kernel-trace only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
K3_SHAPE=${K3_SHAPE:-}
for c in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_k3${K3_TAG}_$i -o k -- python3 scripts/k3_target.py $K3_SHAPE > gpurun_out/pmc_k3${K3_TAG}_$i.log 2>&1 || exit $?
done
export K3_TAG
python3 - <<'PY' > gpurun_out/pmc_k3${K3_TAG}.json && cat gpurun_out/pmc_k3${K3_TAG}.json
import collections, csv, glob, json, os
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/pmc_k3{os.environ.get('K3_TAG', '')}_[0-9]/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "hgnn" in r["Kernel_Name"]:
            acc[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"note": "GRBM_GUI_ACTIVE is summed over the 8 XCDs; mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / "
               "(1024 SIMDs x GRBM_GUI_ACTIVE/8); per-launch means", "kernels": {}}
for k, v in acc.items():
    m = {c: sum(x) / len(x) for c, x in v.items()}
    if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m and m["GRBM_GUI_ACTIVE"]:
        m["mfma_util"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8), 3)
    out["kernels"][k] = m
print(json.dumps(out, indent=1))
PY
