#!/bin/bash
# K3 forward: memory instructions issued inside the sweep (HGNN_XS_VMEM_STEP) — parity tests on
# one variant, k3_xs_bench per variant, phase stamps per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
HGNN_LIB=libhgnn_${TESTLIB:-vm2}.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "linear or k3" > gpurun_out/k3vm_tests.log 2>&1 || { tail -40 gpurun_out/k3vm_tests.log; exit 1; }
tail -1 gpurun_out/k3vm_tests.log
NO_TESTS=1 LIBS="${LIBS:-vm1 vm2 vm4}" TAG=k3vm bash scripts/gpu_r4_ab.sh || exit 1
for v in stamps ${STAMPS:-vmst1 vmst2 vmst4}; do
  echo "== stamps $v"; HGNN_LIB=libhgnn_$v.so timeout -k 10 200 python scripts/k3_stamps.py 2>&1 | grep '^{' || exit 1
done
