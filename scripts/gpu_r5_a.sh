#!/bin/bash
# Round 5, first GPU pass: the parity tests touched by the round's first changes (K3 dispatch
# without the env-only variants, presorted negatives, partial-seed guard, blocked dP gather),
# then the blocked dP gather A/B at cfg4.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "segment_bounds or source_blocks or presorted or dp_gather" \
  > gpurun_out/r5a_tests.log 2>&1 || { tail -30 gpurun_out/r5a_tests.log; exit 1; }
tail -3 gpurun_out/r5a_tests.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_minibatch_graph.py tests/test_capi_gpu.py > gpurun_out/r5a_tests2.log 2>&1 || { tail -30 gpurun_out/r5a_tests2.log; exit 1; }
tail -3 gpurun_out/r5a_tests2.log
timeout -k 10 400 python -u scripts/score_block_bench.py 1:1 8:1 8:0 4:1 12:1 16:1 > gpurun_out/r5a_dp_blocks.jsonl 2>&1 || { tail -20 gpurun_out/r5a_dp_blocks.jsonl; exit 1; }
cat gpurun_out/r5a_dp_blocks.jsonl
