#!/bin/bash
# Round-6 closing pass B: the cfg4 bench line (CPU baseline: median of 3 steps of the 1/8 shard)
# and a rocprofv3 kernel-stats + kernel-trace profile of the same bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r6}
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > gpurun_out/${T}_cfg4.log 2> gpurun_out/${T}_cfg4.err || { tail -20 gpurun_out/${T}_cfg4.err; exit 1; }
grep '^{' gpurun_out/${T}_cfg4.log | tail -1 > gpurun_out/${T}_cfg4_bench_line.json; head -c 400 gpurun_out/${T}_cfg4_bench_line.json; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps > gpurun_out/prof_${T}.log 2>&1 || { tail -5 gpurun_out/prof_${T}.log; exit 1; }
echo "rocprof ok"
