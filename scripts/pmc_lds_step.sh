#!/bin/bash
# LDS bank-conflict cycles per kernel of the cfg4 step (one --pmc pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 400 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_lds -o k -- python3 scripts/pmc_step_target.py cfg4 2 > gpurun_out/pmc_lds.log 2>&1 || { tail -5 gpurun_out/pmc_lds.log; exit 1; }
python3 - <<'PY'
import collections, csv, glob
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for f in glob.glob("gpurun_out/pmc_lds/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
rows = sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_LDS_BANK_CONFLICT", 0))
for k, m in rows[:25]:
    print(f"{k:70s} conf={m.get('SQ_LDS_BANK_CONFLICT',0):.3e} lds={m.get('SQ_INSTS_LDS',0):.3e} gui={m.get('GRBM_GUI_ACTIVE',0):.3e}")
PY
