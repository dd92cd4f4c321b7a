#!/bin/bash
# Targeted GPU tests (-k expression in $K) then the default bench (cfg4), no CPU baseline.
# usage: K="expr" [TESTS="tests/x.py ..."] bash scripts/gpu_quick.sh [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > gpurun_out/gpu_quick_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/gpu_quick_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; python - <<'PY'
import json
for l in open("gpurun_out/bench_quick.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["value"], d["ms_per_step"], {k: v["ms_per_step"] for k, v in d["kernels"].items()})
PY
exit $rc
