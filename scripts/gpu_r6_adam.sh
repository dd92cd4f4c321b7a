#!/bin/bash
# optim.Adam (hgnn_adam_multi): its parity tests and the mini-batch tests that replay it, then
# cfg5 with it against torch's fused Adam (default; ours: --native-adam), A/B on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_adam_matches_torch" tests/test_minibatch_graph.py \
  tests/test_gpu_cfg5_pipeline.py > gpurun_out/adam_tests.log 2>&1 \
  || { tail -30 gpurun_out/adam_tests.log; exit 1; }
tail -2 gpurun_out/adam_tests.log
for v in ${VARIANTS:-torch ours torch ours}; do
  a=""; [ "$v" = ours ] && a="--native-adam"
  timeout -k 10 300 python bench.py --config cfg5 --steps 300 --warmup 20 --no-cpu-baseline --timer-steps 0 $a > gpurun_out/ad.log 2> gpurun_out/ad.err || { tail -5 gpurun_out/ad.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ad.log') if l.startswith('{')][-1]); print('adam', '$v', d['ms_per_step'], repr(d['loss']), d['config']['graph_nodes']['total'])"
done
