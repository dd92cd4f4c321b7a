#!/bin/bash
# cfg5: a rocprofv3 kernel trace of the mini-batch bench, the last ~600 kernels written out with
# their queue (the replay and the sampler's side stream) for scripts/cfg5_trace_nodes.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r6_cfg5}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --config cfg5 --steps 20 --warmup 5 --no-cpu-baseline --profile-steps ${BENCH_ARGS} > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("gpurun_out/prof_$TAG/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-600:]
keys = list(rows[0].keys())
qk = "Queue_Id" if "Queue_Id" in keys else ("Stream_Id" if "Stream_Id" in keys else None)
with open("gpurun_out/${TAG}_trace_tail.csv", "w") as o:
    w = csv.writer(o)
    w.writerow(["start_ns", "dur_ns", "queue", "grid", "name"])
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        w.writerow([s - t0, e - s, r.get(qk, "") if qk else "", r.get("Grid_Size", r.get("Grid_Size_X", "")), r["Kernel_Name"][:140]])
print("columns:", keys)
PY
rm -rf gpurun_out/prof_$TAG
