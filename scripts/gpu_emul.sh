#!/bin/bash
# Per-rank compute of the N-GPU strong-scaled cfg4 step (scripts/shard_emulation.py) under env variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
while IFS= read -r v; do
  echo "== [$v]"
  env $v timeout -k 10 300 python scripts/shard_emulation.py --config ${CFG:-cfg4} --strong --world ${WORLD:-8} --steps 10 > gpurun_out/emul.log 2>&1 || { tail -5 gpurun_out/emul.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/emul.log').read().strip().splitlines()[-1])
print(d['ms_per_step_compute'], d['kernels_sum_ms'])
for k,v in sorted(d['kernels_ms_per_step'].items(), key=lambda kv:-kv[1]): print('   %-42s %7.3f' % (k, v))
"
done <<< "$VARIANTS"
