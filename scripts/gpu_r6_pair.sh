#!/bin/bash
# The K3 pair path (hgnn_linear_{fwd,bwd}_multi): its parity tests, then cfg5 with it off / on and
# the forward's tiles-per-block floor (A/B on one box; HGNN_XS_FWD_TPB was removed after it, the
# floor is 8 now, so only the pair switch still varies).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "linear_multi or fuse_weights_multi or gather_multi" \
  tests/test_minibatch_graph.py tests/test_gpu_cfg5_pipeline.py > gpurun_out/pair_tests.log 2>&1 \
  || { tail -30 gpurun_out/pair_tests.log; exit 1; }
tail -2 gpurun_out/pair_tests.log
for v in ${VARIANTS:-0:1 1:1 0:1 1:1}; do
  p=${v%%:*}; f=${v##*:}
  HGNN_K3_PAIR=$p HGNN_XS_FWD_TPB=$f timeout -k 10 300 python bench.py --config cfg5 --steps 300 --warmup 20 --no-cpu-baseline --timer-steps 0 > gpurun_out/pr.log 2> gpurun_out/pr.err || { tail -5 gpurun_out/pr.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/pr.log') if l.startswith('{')][-1]); print('pair', $p, 'fwd_tpb', $f, d['ms_per_step'], repr(d['loss']), d['config']['graph_nodes']['total'])"
done
