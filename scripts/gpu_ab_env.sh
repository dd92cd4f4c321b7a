#!/bin/bash
# A/B of environment knobs on the default bench (cfg4): one bench run per "VAR=value" argument
# ("-" = no override).  usage: bash scripts/gpu_ab_env.sh "-" "HGNN_STREAMS=1" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
i=0
for kv in "$@"; do
  i=$((i+1))
  if [ "$kv" = "-" ]; then envs=""; else envs="$kv"; fi
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/ab_$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$kv rc=$rc"; tail -5 gpurun_out/ab_$i.log; exit $rc; }
  python3 - "$kv" gpurun_out/ab_$i.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"{sys.argv[1]:40s} {d['ms_per_step']:8.2f} ms/step  timer {d['kernel_timer']['ms_per_step']}")
PY
done
