#!/bin/bash
# Round 6 K3 A/B: the K3 parity tests on the default build and on each variant library in LIBS,
# then scripts/k3_xs_bench.py per library, twice in alternating order (box noise).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-r6k3}
for v in default ${TESTLIBS:-${LIBS}}; do
  if [ $v = default ]; then L=; else L=libhgnn_$v.so; fi
  HGNN_LIB=$L timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "linear or k3" > gpurun_out/${TAG}_tests_$v.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/${TAG}_tests_$v.log)"
done
for rep in 1 2; do
  for v in default ${LIBS}; do
    if [ $v = default ]; then L=; else L=libhgnn_$v.so; fi
    HGNN_LIB=$L timeout -k 10 300 python -u scripts/k3_xs_bench.py ${K3_ARGS} > gpurun_out/${TAG}_k3_${v}_$rep.jsonl 2>&1 || { tail -20 gpurun_out/${TAG}_k3_${v}_$rep.jsonl; exit 1; }
    echo "== $v rep $rep"; python3 -c "
import json
for l in open('gpurun_out/${TAG}_k3_${v}_$rep.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['case'][:40].ljust(40), d['fwd_ms'], d['fwd_frac'], d.get('bwd_ms'), d.get('bwd_frac'), d['fwd_rel_err'])"
  done
done
