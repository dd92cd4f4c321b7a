#!/bin/bash
# Round-2 GPU pass: GPU tests, smoke, default bench (cfg4), rocprofv3 kernel-trace stats of the
# bench.  Each GPU step under its own time limit; stops at the first failure.
# usage: [SKIP_TESTS=1] [PROFILE=tag] bash scripts/gpu_r2.sh [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$PROFILE -o run \
    -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps "$@" > gpurun_out/prof_$PROFILE.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -c 600 gpurun_out/prof_$PROFILE.log
  exit $rc
fi
