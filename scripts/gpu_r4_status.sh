#!/bin/bash
# Round-4 status pass: N = 8 per-rank emulation of the strong-scaled cfg4 step (ranks 0 and 7:
# compute and the collective covers), the cfg5 link-prediction line (with its CPU baseline) and
# the cfg5 replayed path at world 2 (two ranks on the one GPU over gloo).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r4}
for r in 0 7; do
  timeout -k 10 400 python scripts/shard_emulation.py --config cfg4 --strong --world 8 --rank $r > gpurun_out/${TAG}_emul_r$r.log 2>&1 || { tail -20 gpurun_out/${TAG}_emul_r$r.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_emul_r$r.log | tail -1 > gpurun_out/${TAG}_emul_r$r.json
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_emul_r$r.json')); print($r, d['ms_per_step_compute'], d['kernels_sum_ms']); print([(c['op'], c['cover_ms'], c['est_ms_1link_ring'], c['cover_over_1link']) for c in d['collectives']]); print(d['link_timeline']['1link_ring'] if not isinstance(d['link_timeline']['1link_ring'], list) else '')"
done
timeout -k 10 400 python bench.py --config cfg5 --steps 300 --warmup 20 > gpurun_out/${TAG}_cfg5.log 2>&1 || { tail -20 gpurun_out/${TAG}_cfg5.log; exit 1; }
grep '^{' gpurun_out/${TAG}_cfg5.log | tail -1 > gpurun_out/${TAG}_cfg5_bench_line.json; head -c 600 gpurun_out/${TAG}_cfg5_bench_line.json; echo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --config cfg5 --gpus 2 --same-device --dist-backend gloo --steps 50 --warmup 5 > gpurun_out/${TAG}_cfg5_w2.log 2>&1 || { tail -20 gpurun_out/${TAG}_cfg5_w2.log; exit 1; }
grep '^{' gpurun_out/${TAG}_cfg5_w2.log | tail -1 | head -c 700; echo
