#!/bin/bash
# cfg5 mini-batch bench line + a rocprofv3 kernel trace of it (GPU busy time vs wall per step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python bench.py --config cfg5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/cfg5_bench.log 2>&1 || { tail -5 gpurun_out/cfg5_bench.log; exit 1; }
grep '^{' gpurun_out/cfg5_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('cfg5', d['ms_per_step'], d['value'], d['config']['batches_per_s'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_cfg5 -o run -- python3 bench.py --config cfg5 --steps 20 --warmup 5 --no-cpu-baseline --profile-steps > gpurun_out/prof_cfg5.log 2>&1 || { tail -5 gpurun_out/prof_cfg5.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_cfg5/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-400:]
t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
print(f"last {len(rows)} kernels: wall {(t1-t0)/1e6:.2f} ms, busy {busy/1e6:.2f} ms")
PY
