#!/bin/bash
# Per-kernel times of the negatives sort at cfg4 size (scripts/sort_bench.py under rocprofv3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sortprof -o run -- python3 scripts/sort_bench.py "$@" > gpurun_out/sortprof.log 2>&1 || { tail -20 gpurun_out/sortprof.log; exit 1; }
cat gpurun_out/sortprof.log | grep -v amdgpu.ids
python3 - gpurun_out/sortprof/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'hgnn' in r['Name'] or 'uniform' in r['Name']: print(r['Name'][:90], r['Calls'], r['AverageNs'])
PY
