#!/bin/bash
# Round 5, third pass: sort A/B (leader-read scatter) and K3 A/B (cheaper mask bits) on variant
# libraries, each with its parity tests first.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
LIBS=leader NO_TESTS= bash scripts/gpu_sort_ab.sh || exit 1
HGNN_LIB=libhgnn_maskmed.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "linear or k3" > gpurun_out/r5c_k3_tests_maskmed.log 2>&1 || { tail -40 gpurun_out/r5c_k3_tests_maskmed.log; exit 1; }
tail -1 gpurun_out/r5c_k3_tests_maskmed.log
NO_TESTS=1 LIBS=maskmed TAG=r5c bash scripts/gpu_r4_ab.sh
