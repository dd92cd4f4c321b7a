#!/bin/bash
# Round 4: K3 split-once kernels — parity tests of every K3 family, then the cfg4-shape A/B.
set -o pipefail
mkdir -p gpurun_out
./tmp_probe/med_probe && timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "linear or k3" > gpurun_out/r4_k3_tests.log 2>&1 || { tail -40 gpurun_out/r4_k3_tests.log; exit 1; }
tail -3 gpurun_out/r4_k3_tests.log
timeout -k 10 240 python -u scripts/k3_xs_bench.py ${K3_ONLY:+--only "$K3_ONLY"} > gpurun_out/r4_k3_xs.jsonl 2>&1 || { tail -20 gpurun_out/r4_k3_xs.jsonl; exit 1; }
cat gpurun_out/r4_k3_xs.jsonl
