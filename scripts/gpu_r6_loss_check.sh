#!/bin/bash
# cfg5: the pipelined bench (next batch staged on a side stream; by default two recorded steps
# in turn) against the unpipelined and single-buffer ones — the same batches and steps, so the
# end-of-run loss must agree bitwise.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
run() {
  timeout -k 10 300 python bench.py --config cfg5 --steps ${STEPS:-300} --warmup 20 --no-cpu-baseline --timer-steps 0 "$@" > gpurun_out/lc.log 2> gpurun_out/lc.err || { tail -5 gpurun_out/lc.err; exit 1; }
  python3 -c "import json, os; d=json.loads([l for l in open('gpurun_out/lc.log') if l.startswith('{')][-1]); print('$*', d['ms_per_step'], repr(d['loss']), d['config'].get('recorded_steps'))"
}
run
run --single-buffer
run --no-prefetch
