#!/bin/bash
# Full-size parity + new golden tests, then the cfg4 step PMC passes and K3 PMC at cfg4 shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_full_size.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "full_size or fused_loss or golden or second_backward" > gpurun_out/gpu_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/gpu_full.log | tail -40
[ $rc -eq 0 ] || exit $rc
bash scripts/pmc_r2.sh || exit $?
K3_SHAPE="9000000 128 128" K3_TAG=_cfg4 bash scripts/pmc_k3.sh > gpurun_out/pmc_k3_cfg4.out 2>&1 || exit $?
echo k3 ok
