#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 400 python scripts/sampler_bench.py > gpurun_out/sampler.log 2>&1; rc=$?; tail -2 gpurun_out/sampler.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 scripts/sampler_bench.py --scale 0.1 > gpurun_out/sampler_dist1.log 2>&1; rc=$?; tail -1 gpurun_out/sampler_dist1.log; exit $rc
