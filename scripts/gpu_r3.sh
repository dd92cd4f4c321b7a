#!/bin/bash
# Round-3 GPU pass.  Each GPU step under its own time limit; stops at the first failure.
# usage: [TESTS="<pytest args>"] [SKIP_BENCH=1] [PROFILE=tag] bash scripts/gpu_r3.sh [bench args...]
#   TESTS unset: the whole -m gpu suite + smoke; TESTS=none: no tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-all}" != "none" ]; then
  if [ "${TESTS:-all}" = "all" ]; then T="tests -m gpu"; else T="$TESTS"; fi
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $T -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -8
  [ $rc -eq 0 ] || { tail -60 gpurun_out/gpu_tests.log; exit $rc; }
  if [ "${TESTS:-all}" = "all" ]; then
    timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
    [ $rc -eq 0 ] || exit $rc
  fi
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$PROFILE -o run \
    -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps "$@" > gpurun_out/prof_$PROFILE.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -c 600 gpurun_out/prof_$PROFILE.log
  exit $rc
fi
