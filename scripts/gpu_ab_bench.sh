#!/bin/bash
# GPU tests, then bench A/B over an environment switch: ENVA / ENVB (e.g. HGNN_PREPROJECT=0 / 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for e in "$ENVA" "$ENVB"; do
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1
  rc=$?; echo "[$e] bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/ab.log; exit $rc; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['value'])
for k,v in sorted(d['kernels'].items(), key=lambda kv:-kv[1]['ms_per_step']): print('   %-45s %8.3f' % (k, v['ms_per_step']))
"
done
