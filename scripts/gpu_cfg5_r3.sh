#!/bin/bash
# cfg5 mini-batch: bench A/B of the side-stream prefetch of the next batch, and a rocprofv3
# kernel trace of the prefetching bench (GPU busy = the union of kernel intervals over the last
# 400 kernels, against their wall span).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rep in 1 2; do
  for pf in "" "--no-prefetch"; do
    timeout -k 10 300 python bench.py --config cfg5 --steps 200 --warmup 20 --no-cpu-baseline --timer-steps 0 $pf > gpurun_out/cfg5_bench.log 2>&1 || { tail -5 gpurun_out/cfg5_bench.log; exit 1; }
    grep '^{' gpurun_out/cfg5_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('cfg5 $pf', d['ms_per_step'], d['value'], d['config']['batches_per_s'])"
  done
done
timeout -k 10 300 python bench.py --config cfg5 --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/cfg5_bench_line.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_cfg5 -o run -- python3 bench.py --config cfg5 --steps 40 --warmup 10 --no-cpu-baseline --profile-steps --prefetch > gpurun_out/prof_cfg5.log 2>&1 || { tail -5 gpurun_out/prof_cfg5.log; exit 1; }
python3 - <<'PY'
import csv, glob, json
f = glob.glob("gpurun_out/prof_cfg5/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-400:]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
busy, cur_s, cur_e = 0, None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
wall = iv[-1][1] - iv[0][0]
print(json.dumps({"kernels": len(rows), "wall_ms": round(wall / 1e6, 3), "busy_ms": round(busy / 1e6, 3),
                  "busy_frac": round(busy / wall, 3)}))
PY
