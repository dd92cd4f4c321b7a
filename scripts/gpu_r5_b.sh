#!/bin/bash
# Round 5, second pass: the captured RCCL all-reduce test, the mini-batch graph tests, the
# distributed GPU tests on the new default last-gather chunking, and the N = 8 emulation.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_minibatch_graph.py tests/test_gpu_dist.py > gpurun_out/r5b_tests.log 2>&1 || { tail -40 gpurun_out/r5b_tests.log; exit 1; }
tail -3 gpurun_out/r5b_tests.log
timeout -k 10 300 python bench.py --config cfg5 --dist --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r5b_cfg5_dist_w1.log 2>&1 || { tail -30 gpurun_out/r5b_cfg5_dist_w1.log; exit 1; }
grep '^{' gpurun_out/r5b_cfg5_dist_w1.log | tail -1 > gpurun_out/r5b_cfg5_dist_w1.json; head -c 900 gpurun_out/r5b_cfg5_dist_w1.json; echo
MODES="${MODES:-3:2:1 3:2:2}" RANKS="0 3 7" bash scripts/gpu_r5_emul.sh
