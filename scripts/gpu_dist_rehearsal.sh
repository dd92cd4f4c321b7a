#!/bin/bash
# N=2 bench rehearsal on one GPU (gloo over device tensors): the sharded bench path end to end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --same-device --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rehearsal_w2.log 2>&1; rc=$?
tail -1 gpurun_out/rehearsal_w2.log | cut -c1-900; exit $rc
