#!/bin/bash
# Quick GPU pass: selected tests (-k expr in $1), then bench at N=1 (extra args after $1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
K="$1"; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu -k "$K" > gpurun_out/quick_tests.log 2>&1; rc=$?; tail -4 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/quick_bench.log 2>&1; rc=$?; tail -1 gpurun_out/quick_bench.log | head -c 700; echo; exit $rc
