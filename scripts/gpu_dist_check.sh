#!/bin/bash
# Sharded path on one GPU: dist tests (gloo over device tensors, RCCL-path adjoints forced), the
# world-2 bench rehearsal, and the RCCL world-1 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_parity.py -k "shard or halo" > gpurun_out/dist_tests.log 2>&1; rc=$?; tail -6 gpurun_out/dist_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --same-device --dist-backend gloo --config cfg5 --scale 0.02 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_cfg5_w2.log 2>&1; rc=$?; tail -1 gpurun_out/b_cfg5_w2.log | cut -c1-300; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dist --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_dist1.log 2>&1; rc=$?; tail -1 gpurun_out/b_dist1.log | cut -c1-300; echo; exit $rc
