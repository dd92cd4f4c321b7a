#!/bin/bash
# bench at N=1 only (kernel table), optional -k tests first: bash scripts/gpu_quick_bench.sh "<k expr>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
if [ -n "$1" ]; then
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu -k "$1" > gpurun_out/quick_tests.log 2>&1; rc=$?; tail -2 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/quick_bench.log 2>&1 || exit 1
python - <<'PY'
import json
l = json.loads(open("gpurun_out/quick_bench.log").read().strip().splitlines()[-1])
print("ms/step", l["ms_per_step"], "edges/s %.4g" % l["value"], "roof", l["roofline"]["frac"])
for k, v in sorted(l["kernels"].items(), key=lambda x: -x[1]["ms_per_step"]):
    print(f"  {v['ms_per_step']:7.3f} {v['GB/s']:9.1f} {k}")
PY
