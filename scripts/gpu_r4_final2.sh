#!/bin/bash
# Round-4 second closing pass: the whole -m gpu suite + smoke, the cfg4 bench line with its CPU
# baseline, a rocprofv3 kernel-stats profile of the same bench, the N = 8 emulation (ranks 0, 7).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r4g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/${T}_gpu_tests.log; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > gpurun_out/${T}_cfg4.log 2> gpurun_out/${T}_cfg4.err || { tail -20 gpurun_out/${T}_cfg4.err; exit 1; }
grep '^{' gpurun_out/${T}_cfg4.log | tail -1 > gpurun_out/${T}_cfg4_bench_line.json; head -c 300 gpurun_out/${T}_cfg4_bench_line.json; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps > gpurun_out/prof_${T}.log 2>&1 || { tail -5 gpurun_out/prof_${T}.log; exit 1; }
echo "rocprof ok"
for r in 0 7; do
  timeout -k 10 400 python scripts/shard_emulation.py --config cfg4 --strong --world 8 --rank $r > gpurun_out/${T}_emul_r$r.log 2>&1 || { tail -20 gpurun_out/${T}_emul_r$r.log; exit 1; }
  grep '^{' gpurun_out/${T}_emul_r$r.log | tail -1 > gpurun_out/${T}_emul_r$r.json
done
echo "emulation ok"
