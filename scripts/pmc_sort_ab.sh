#!/bin/bash
# LDS bank-conflict cycles of the negatives sort (scripts/sort_bench.py --mode draw, cfg4 sizes)
# per variant library: LIBS="lanehist" (default build first).  One --pmc pass per library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default ${LIBS}; do
  if [ $v = default ]; then L=; else L=libhgnn_$v.so; fi
  HGNN_LIB=$L timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sort_$v -o k -- python3 scripts/sort_bench.py --mode draw --reps 3 > gpurun_out/pmc_sort_$v.log 2>&1 || { tail -5 gpurun_out/pmc_sort_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import collections, csv, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(f"gpurun_out/pmc_sort_{sys.argv[1]}/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "digit" not in r["Kernel_Name"]: continue
        k = r["Kernel_Name"].split("(")[0].replace("void hgnn::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, m in sorted(acc.items()):
    c, l, w = m.get("SQ_LDS_BANK_CONFLICT", 0), m.get("SQ_INSTS_LDS", 1), m.get("SQ_WAVE_CYCLES", 1)
    print(f"{sys.argv[1]:9s} {k:45s} conflict/LDS-instr={c / l:6.2f} conflict/wave-cycles={c / (4 * w):.3f}")
PY
done
