#!/bin/bash
# K1 source-block slice A/B at cfg4 on the final build: HGNN_GATHER_BLOCK_MB (600 -> 8 passes over
# the 4.6 GB user table; 660 -> 7, 520 -> 9, 460 -> 10).  Step time, the roofline launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for mb in ${MBS:-600 660 520 460}; do
  HGNN_GATHER_BLOCK_MB=$mb timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/k1b_$mb.log 2>&1 || { tail -5 gpurun_out/k1b_$mb.log; exit 1; }
  grep '^{' gpurun_out/k1b_$mb.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']
print('$mb MB', d['ms_per_step'], 'K1 us', r['avg_launch_us'], 'frac', r['frac'])"
done
