#!/bin/bash
# Where the bf16x6 K3 kernels' cycles go at the cfg4 user-side shapes (K = 128, 256): MFMA busy,
# LDS bank conflicts, instruction mix and wave-cycle breakdown.  Separate --pmc passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for shape in "9000000 64 128" "9000000 128 128"; do
  tag=k$(( $(echo $shape | cut -d' ' -f2) * 2 ))
  i=0
  for c in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmcx6_${tag}_$i -o k -- python3 scripts/k3_target.py $shape > gpurun_out/pmcx6_${tag}_$i.log 2>&1 || { echo "pass $tag/$i rc=$?"; tail -3 gpurun_out/pmcx6_${tag}_$i.log; exit 1; }
  done
done
python3 - <<'PY' > gpurun_out/pmc_k3_cfg4_r3.json && cat gpurun_out/pmc_k3_cfg4_r3.json
import collections, csv, glob, json
out = {"note": "cfg4 user-side shapes, N = 9M rows, H = 128 (scripts/k3_target.py: 5 backward + 5 "
               "forward launches); per-launch means; GRBM_GUI_ACTIVE is summed over the 8 XCDs, "
               "mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)",
       "shapes": {}}
for tag in ("k128", "k256"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/pmcx6_{tag}_[0-9]/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "hgnn" in r["Kernel_Name"]:
                acc[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    ks = {}
    for k, v in acc.items():
        m = {c: sum(x) / len(x) for c, x in v.items()}
        if m.get("GRBM_GUI_ACTIVE"):
            m["mfma_util"] = round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * m["GRBM_GUI_ACTIVE"] / 8), 3)
        ks[k] = {c: (round(x, 3) if isinstance(x, float) and x < 10 else round(x)) for c, x in m.items()}
    out["shapes"][tag] = ks
print(json.dumps(out, indent=1))
PY
