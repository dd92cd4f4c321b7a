#!/bin/bash
# cfg5 with the side stream's sampling confined to N CUs (a CU-masked stream), A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for n in ${CUS:-0 32 64 128 0 32 64}; do
  timeout -k 10 300 python bench.py --config cfg5 --steps 300 --warmup 20 --no-cpu-baseline --timer-steps 0 --side-cus $n > gpurun_out/cus.log 2> gpurun_out/cus.err || { tail -5 gpurun_out/cus.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/cus.log') if l.startswith('{')][-1]); print('side_cus', $n, d['ms_per_step'], repr(d['loss']))"
done
