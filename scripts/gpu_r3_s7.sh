#!/bin/bash
# A/B: conflict-free LDS layouts of the bf16x6 K3 kernels (libhgnn_base.so = before), K3 parity
# tests, cfg4 bench both ways, and the bank-conflict counter of the new build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "linear or k3 or golden or step" > gpurun_out/t7.log 2>&1 || { tail -30 gpurun_out/t7.log; exit 1; }
tail -1 gpurun_out/t7.log
for rep in 1 2; do
  for lib in libhgnn_base.so libhgnn.so; do
    echo "== $lib"
    HGNN_LIB=$lib timeout -k 10 120 python scripts/k3_ab.py --rows 9000000 --k 128 --add --bwd || exit 1
    HGNN_LIB=$lib timeout -k 10 120 python scripts/k3_ab.py --rows 9000000 --k 256 --segs 2 --bwd || exit 1
    HGNN_LIB=$lib timeout -k 10 120 python scripts/k3_ab.py --rows 1000000 --k 256 --segs 2 --bwd || exit 1
  done
done
for lib in libhgnn_base.so libhgnn.so; do
  HGNN_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b7_$lib.log 2>&1 || { tail -20 gpurun_out/b7_$lib.log; exit 1; }
  echo "$lib"; grep '^{' gpurun_out/b7_$lib.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'linear' in n})"
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc7 -o k -- python3 scripts/k3_target.py 9000000 128 128 > gpurun_out/pmc7.log 2>&1 || { tail -3 gpurun_out/pmc7.log; exit 1; }
python3 - <<'PY'
import collections, csv, glob
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc7/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "x6" in r["Kernel_Name"]:
            acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    m = {c: sum(x) / len(x) for c, x in v.items()}
    m["mfma_util"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
    print(k, {c: round(x, 3) for c, x in m.items()})
PY
