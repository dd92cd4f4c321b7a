#!/bin/bash
# Round-6 closing pass A: the whole -m gpu suite and smoke on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r6}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/${T}_gpu_tests.log | head; tail -40 gpurun_out/${T}_gpu_tests.log; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
