#!/bin/bash
# cfg5 step phases (bench.py HGNN_CFG5_PHASES=1): host time per loop phase and GPU spans per batch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r6ph}
for v in ${VARIANTS:-default}; do
  extra=""; [ "$v" != default ] && extra="$v"
  HGNN_CFG5_PHASES=1 timeout -k 10 300 python bench.py --config cfg5 --steps 200 --warmup 20 --no-cpu-baseline --timer-steps 0 $extra > gpurun_out/${T}.log 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/${T}.log') if l.startswith('{')][-1]); print('$v', d['ms_per_step'], json.dumps(d.get('phases')))"
done
