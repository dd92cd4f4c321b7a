#!/bin/bash
# K3 A/B over variant libraries (scripts/build_variant.py): parity tests of every K3 family on the
# default build, then scripts/k3_xs_bench.py per library.   LIBS="s0 p1" (default build first).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-ab}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "linear or k3" > gpurun_out/${TAG}_k3_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_k3_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_k3_tests.log
fi
for v in default ${LIBS}; do
  if [ $v = default ]; then L=; else L=libhgnn_$v.so; fi
  HGNN_LIB=$L timeout -k 10 300 python -u scripts/k3_xs_bench.py ${K3_ARGS} > gpurun_out/${TAG}_k3_$v.jsonl 2>&1 || { tail -20 gpurun_out/${TAG}_k3_$v.jsonl; exit 1; }
  echo "== $v"; python3 -c "
import json
for l in open('gpurun_out/${TAG}_k3_$v.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['case'][:40].ljust(40), d['fwd_ms'], d['fwd_frac'], d['bwd_ms'], d['bwd_frac'])"
done
