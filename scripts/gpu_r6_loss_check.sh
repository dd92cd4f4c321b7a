#!/bin/bash
# cfg5: the pipelined bench (next batch staged on a side stream) against the unpipelined one —
# the same batches and steps, so the end-of-run loss must agree bitwise — and, with
# HGNN_CFG5_SERIAL=1 (every step synchronised), the first per-step losses, the parameters after
# the capture and the staged batch 0's checksums of both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
run() {
  timeout -k 10 300 python bench.py --config cfg5 --steps ${STEPS:-300} --warmup 20 --no-cpu-baseline --timer-steps 0 "$@" > gpurun_out/lc.log 2> gpurun_out/lc.err || { tail -5 gpurun_out/lc.err; exit 1; }
  python3 -c "import json, os; d=json.loads([l for l in open('gpurun_out/lc.log') if l.startswith('{')][-1]); print(os.environ.get('HGNN_CFG5_SERIAL', '0'), '$*', d['ms_per_step'], repr(d['loss']), d.get('losses', [])[:4], d.get('after_capture'))"
}
run
run --no-prefetch
run --eager-sampler
