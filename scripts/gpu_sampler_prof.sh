#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof -o run -- python scripts/sampler_bench.py --batches 10 > gpurun_out/sprof.log 2>&1; rc=$?; tail -1 gpurun_out/sprof.log; exit $rc
