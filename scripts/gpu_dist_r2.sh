#!/bin/bash
# Rehearsal of bench.py's multi-rank paths on a 1-GPU box (8-GPU runs are the driver's):
#  1. the spawn launcher (`bench.py --gpus N` without torch.distributed.run) with N ranks on cuda:0
#     over gloo (device tensors), strong-scaled cfg4 shrunk;
#  2. world 1 through RCCL (--dist) at full cfg4: the sharded step's setup, memory and time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --gpus 2 --same-device --dist-backend gloo --scale 0.05 --steps 3 --warmup 1 --timer-steps 2 > gpurun_out/dist_n2.log 2>&1
rc=$?; echo "n2 rc=$rc"; tail -c 1500 gpurun_out/dist_n2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 8 --same-device --dist-backend gloo --scale 0.02 --steps 2 --warmup 1 --timer-steps 1 > gpurun_out/dist_n8.log 2>&1
rc=$?; echo "n8 rc=$rc"; tail -c 600 gpurun_out/dist_n8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --dist --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/dist_w1_rccl.log 2>&1
rc=$?; echo "w1 rccl rc=$rc"; tail -c 2500 gpurun_out/dist_w1_rccl.log; [ $rc -eq 0 ] || exit $rc
