#!/bin/bash
# Round 5: per-rank compute of the strong-scaled cfg4 step at N = 2 and 4 (first and last rank),
# with the closing build's defaults, beside the N = 8 runs of gpu_r5_emul.sh: the predicted
# 1/2/4/8 curve (compute per rank, one-link stall) for the driver's scaling run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r5}
for wr in ${WORLDS:-2:0 2:1 4:0 4:3}; do
  IFS=: read w r <<< "$wr"
  out=gpurun_out/${TAG}_emul_n${w}_r$r
  timeout -k 10 400 python scripts/shard_emulation.py --config cfg4 --strong --world $w --rank $r --steps 10 > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
  grep '^{' $out.log | tail -1 > $out.json
  python -c "import json; d=json.load(open('$out.json')); t=d['link_timeline']['1link_ring']; print('$w', $r, d['ms_per_step_compute'], 'stall', t['stall_ms'])"
done
