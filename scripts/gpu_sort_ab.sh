#!/bin/bash
# Negatives-sort A/B over variant libraries (scripts/build_variant.py): the sort tests on each, then
# scripts/sort_bench.py (cfg4: 200M draws over 1M posts) per digit width.   LIBS="..." (default
# build first), BITS="0 8 10" (0: the planner's choice; else HGNN_SORT_BITS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in default ${LIBS}; do
  if [ $v = default ]; then L=; else L=libhgnn_$v.so; fi
  HGNN_LIB=$L timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "sort or negative or csr" > gpurun_out/sortab_tests_$v.log 2>&1 || { tail -30 gpurun_out/sortab_tests_$v.log; exit 1; }
  echo "== $v $(tail -1 gpurun_out/sortab_tests_$v.log)"
  for bits in ${BITS:-0}; do
    echo "-- bits $bits"
    HGNN_SORT_BITS=$bits HGNN_LIB=$L timeout -k 10 200 python -u scripts/sort_bench.py --mode draw ${SORT_ARGS} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
