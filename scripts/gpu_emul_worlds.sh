#!/bin/bash
# Per-rank compute of the strong-scaled cfg4 sharded step at N = 1, 2, 4, 8 (scripts/shard_emulation.py;
# collectives stubbed) -> profiles-ready JSON lines in gpurun_out/emul_n*.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for w in ${WORLDS:-1 2 4 8}; do
  timeout -k 10 300 python scripts/shard_emulation.py --config ${CFG:-cfg4} --strong --world $w --steps 10 > gpurun_out/emul_n$w.log 2>&1 || { tail -5 gpurun_out/emul_n$w.log; exit 1; }
  tail -1 gpurun_out/emul_n$w.log > gpurun_out/emul_n$w.json
  python3 -c "
import json; d=json.load(open('gpurun_out/emul_n$w.json')); print($w, d['ms_per_step_compute'], d['kernels_sum_ms'])"
done
