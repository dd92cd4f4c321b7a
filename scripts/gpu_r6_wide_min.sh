#!/bin/bash
# cfg5: the K = 384 blocks below N rows on the general K3 kernels instead of the split pair (A/B;
# the HGNN_XS_WIDE_MIN_ROWS switch it set was removed once the pair path made 0 the better value).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for n in ${MINS:-0 8192 0 8192 65536}; do
  HGNN_XS_WIDE_MIN_ROWS=$n timeout -k 10 300 python bench.py --config cfg5 --steps 300 --warmup 20 --no-cpu-baseline --timer-steps 0 > gpurun_out/wm.log 2> gpurun_out/wm.err || { tail -5 gpurun_out/wm.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/wm.log') if l.startswith('{')][-1]); print('wide_min_rows', $n, d['ms_per_step'], repr(d['loss']), d['config']['graph_nodes']['total'])"
done
