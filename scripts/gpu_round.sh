#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, optional rocprofv3 kernel-trace summary.
# Stops at the first fault/abort/timeout (only pytest's "tests failed" rc=1 continues).
# usage: [PROFILE=tag] [SKIP_TESTS=1] bash scripts/gpu_round.sh [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
  ok $rc || exit $rc
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
  ok $rc || exit $rc
fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$PROFILE -o run \
    -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps > gpurun_out/prof_$PROFILE.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof_$PROFILE.log
  exit $rc
fi
