#!/bin/bash
# N = 8 per-rank compute of the strong-scaled cfg4 step with the closing build (ranks 0 and 7).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 0 7; do
  timeout -k 10 400 python scripts/shard_emulation.py --config cfg4 --strong --world 8 --rank $r > gpurun_out/emul_r$r.log 2>&1 || { tail -20 gpurun_out/emul_r$r.log; exit 1; }
  grep '^{' gpurun_out/emul_r$r.log | tail -1 > gpurun_out/emul_r$r.json; python -c "import json; d=json.load(open('gpurun_out/emul_r$r.json')); print($r, d['ms_per_step_compute'], d['kernels_sum_ms'])"
done
