#!/bin/bash
# Sharded-step schedule changes: HIP-kernel distributed tests, the spawn launcher rehearsal (gloo,
# one device), world-1 RCCL cfg4, and the per-rank emulation at N = 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_dist_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gpu_dist_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 2 --same-device --dist-backend gloo --scale 0.05 --steps 3 --warmup 1 --timer-steps 2 > gpurun_out/dist_n2.log 2>&1
rc=$?; echo "n2 rc=$rc"; [ $rc -eq 0 ] || { tail -c 1500 gpurun_out/dist_n2.log; exit $rc; }
timeout -k 10 400 python bench.py --dist --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/dist_w1_rccl.log 2>&1
rc=$?; echo "w1 rccl rc=$rc"; [ $rc -eq 0 ] || { tail -c 1500 gpurun_out/dist_w1_rccl.log; exit $rc; }
python3 -c "
import json
for f in ['gpurun_out/dist_n2.log','gpurun_out/dist_w1_rccl.log']:
    for l in open(f):
        if l.startswith('{'): d=json.loads(l); print(f, d['n_gpus'], d['ms_per_step'], d['loss'])"
WORLDS=8 bash scripts/gpu_emul_worlds.sh
