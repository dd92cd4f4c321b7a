#!/bin/bash
# Round-6 secondary bench lines: cfg5 (sampled link mini-batches, CPU baseline on one batch's
# blocks), cfg2, cfg3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r6}
for c in ${CONFIGS:-cfg5 cfg2 cfg3}; do
  extra=""; [ $c = cfg5 ] && extra="--steps 200 --warmup 20"
  timeout -k 10 600 python bench.py --config $c $extra > gpurun_out/${T}_$c.log 2> gpurun_out/${T}_$c.err || { tail -20 gpurun_out/${T}_$c.err; exit 1; }
  grep '^{' gpurun_out/${T}_$c.log | tail -1 > gpurun_out/${T}_${c}_bench_line.json
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_${c}_bench_line.json')); print('$c', d['ms_per_step'], d['value'], (d.get('cpu_baseline') or {}).get('value'))"
done
