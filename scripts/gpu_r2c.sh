#!/bin/bash
# Sharded-step pre-projection: the HIP-kernel distributed tests, then the world-1 RCCL sharded
# bench at full cfg4 (the N>1 code path on one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_dist_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_dist_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --dist --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/dist_w1_rccl.log 2>&1
rc=$?; echo "w1 rccl rc=$rc"; tail -c 300 gpurun_out/dist_w1_rccl.log; [ $rc -eq 0 ] || exit $rc
