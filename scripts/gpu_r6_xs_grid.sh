#!/bin/bash
# cfg5: the split K3 kernels' grid as at least F (forward) / B (backward) tiles per block (A/B;
# the HGNN_XS_*_TPB knobs it set were removed after it: the forward keeps a floor of 8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in ${VARIANTS:-1:1 1:8 1:12 1:16 4:1 8:1 1:1 4:12}; do
  f=${v%%:*}; b=${v##*:}
  HGNN_XS_FWD_TPB=$f HGNN_XS_BWD_TPB=$b timeout -k 10 300 python bench.py --config cfg5 --steps 300 --warmup 20 --no-cpu-baseline --timer-steps 0 > gpurun_out/xg.log 2> gpurun_out/xg.err || { tail -5 gpurun_out/xg.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/xg.log') if l.startswith('{')][-1]); print('fwd_tpb', $f, 'bwd_tpb', $b, d['ms_per_step'], repr(d['loss']), d['config']['graph_nodes']['total'])"
done
