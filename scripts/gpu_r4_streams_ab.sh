#!/bin/bash
# A/B of HGNN_STREAMS (independent destination types on two HIP streams) on the final build, cfg4,
# alternating on one box.  Usage (on the GPU box): bash scripts/gpu_r4_streams_ab.sh
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for s in 0 1; do
    HGNN_STREAMS=$s timeout -k 10 420 python bench.py --config cfg4 --steps 10 --warmup 3 \
      --no-cpu-baseline --timer-steps 1 > gpurun_out/r4s_s${s}_${rep}.log 2>&1 || exit 1
    python3 -c "import json,sys; l=[x for x in open('gpurun_out/r4s_s${s}_${rep}.log') if x.startswith('{')][-1]; d=json.loads(l); print('streams=$s rep=$rep', d['ms_per_step'], d['loss'])"
  done
done
