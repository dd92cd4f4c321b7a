#!/bin/bash
# Where the K3 forward's cycles go: wave-cycle breakdown counters for v4 and v5 at the cfg4 shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 4 5; do
  i=0
  for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC" "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES"; do
    i=$((i+1))
    HGNN_K3_FWD=$v HGNN_K3_DGRAD=$v timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_stall_v${v}_$i -o k -- python3 scripts/k3_target.py 9000000 128 128 > gpurun_out/pmc_stall_v${v}_$i.log 2>&1 || echo "pass $v/$i rc=$?"
  done
done
python3 - <<'PY'
import collections, csv, glob, json
for v in (4, 5):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/pmc_stall_v{v}_[0-9]/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "hgnn" in r["Kernel_Name"]:
                acc[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, m in acc.items():
        print(v, k, {c: round(sum(x) / len(x)) for c, x in m.items()})
PY
