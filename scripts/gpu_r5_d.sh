#!/bin/bash
# Round 5: multi-rank rehearsals on one GPU (spawned N = 2 / 8 over gloo, world 1 over RCCL at
# full cfg4) and the cfg2 / cfg3 / cfg5 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/gpu_dist_r2.sh > gpurun_out/r5_dist.txt 2>&1 || { tail -30 gpurun_out/r5_dist.txt; exit 1; }
grep "rc=" gpurun_out/r5_dist.txt
for c in cfg2 cfg3; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 > gpurun_out/r5_$c.log 2>&1 || { tail -20 gpurun_out/r5_$c.log; exit 1; }
  grep '^{' gpurun_out/r5_$c.log | tail -1 > gpurun_out/r5_${c}_bench_line.json; head -c 250 gpurun_out/r5_${c}_bench_line.json; echo
done
timeout -k 10 400 python bench.py --config cfg5 --steps 300 --warmup 20 > gpurun_out/r5_cfg5.log 2>&1 || { tail -20 gpurun_out/r5_cfg5.log; exit 1; }
grep '^{' gpurun_out/r5_cfg5.log | tail -1 > gpurun_out/r5_cfg5_bench_line.json; head -c 250 gpurun_out/r5_cfg5_bench_line.json; echo
