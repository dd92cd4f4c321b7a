#!/bin/bash
# Sort tests, the negatives-sort microbench, then the multi-rank rehearsal of the closing build
# (scripts/gpu_dist_r2.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_edges.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "sort or draw or csr or coo" > gpurun_out/t6.log 2>&1 || { tail -30 gpurun_out/t6.log; exit 1; }
tail -1 gpurun_out/t6.log
timeout -k 10 120 python scripts/sort_bench.py --mode draw || exit 1
bash scripts/gpu_dist_r2.sh
