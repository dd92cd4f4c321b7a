#!/bin/bash
# Round-6 cfg5 iteration: the mini-batch graph tests, the cfg5 bench line, then the replay trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r6c5}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_minibatch_graph.py ${TESTS} > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 400 python bench.py --config cfg5 --steps 300 --warmup 20 ${BENCH_ARGS} > gpurun_out/${T}_cfg5.log 2> gpurun_out/${T}_cfg5.err || { tail -20 gpurun_out/${T}_cfg5.err; exit 1; }
grep '^{' gpurun_out/${T}_cfg5.log | tail -1 > gpurun_out/${T}_cfg5_bench_line.json
python3 -c "import json; d=json.load(open('gpurun_out/${T}_cfg5_bench_line.json')); print('cfg5', d['ms_per_step'], d['value'], (d.get('cpu_baseline') or {}).get('value'))"
[ -n "$NO_TRACE" ] || TAG=${T} bash scripts/gpu_r6_cfg5_trace.sh
