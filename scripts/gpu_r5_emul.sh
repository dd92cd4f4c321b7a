#!/bin/bash
# Round 5: the N = 8 per-rank emulation of the strong-scaled cfg4 step (ranks 0, 3 and 7) for
# the last forward gather's dP chunking modes: one-link stall and covers per collective.
# MODES="3:2:1 2:2:1 3:3:2" (HGNN_CHUNKED_GATHER:HGNN_CHUNK_GROUP:HGNN_CHUNK_FIRST), RANKS="0 7", TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r5}
for m in ${MODES:-3:2 2:2}; do
  for r in ${RANKS:-0 7}; do
    IFS=: read mode grp first <<< "$m"
    out=gpurun_out/${TAG}_emul_m${mode}g${grp}f${first}_r$r
    HGNN_CHUNKED_GATHER=$mode HGNN_CHUNK_GROUP=$grp HGNN_CHUNK_FIRST=${first:-1} timeout -k 10 400 \
      python scripts/shard_emulation.py --config cfg4 --strong --world 8 --rank $r --steps 10 > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
    grep '^{' $out.log | tail -1 > $out.json
    python -c "import json; d=json.load(open('$out.json')); t=d['link_timeline']['1link_ring']; print('$m', $r, d['ms_per_step_compute'], 'stall', t['stall_ms'], t['stall_ms_by_collective'])"
  done
done
