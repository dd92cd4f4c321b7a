#!/bin/bash
# Round-4 closing pass (one GPU call): the whole -m gpu suite + smoke, PMC traffic of the cfg4
# step (-> profiles/pmc_r4.json), the K3 PMC passes, the cfg4 bench line with its CPU baseline, a
# rocprofv3 kernel-stats profile of the same bench, cfg2 / cfg3 / cfg5 lines.  Each GPU step under
# its own time limit; stops at the first failure.   TAG=... names the outputs (default r4f).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r4f}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/${T}_gpu_tests.log; exit $rc; }
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }
  tail -1 gpurun_out/${T}_smoke.log
fi
bash scripts/pmc_r2.sh || exit $?
cp gpurun_out/pmc_step_cfg4.json gpurun_out/${T}_pmc_step_cfg4.json
TAG=$T bash scripts/pmc_k3_xs.sh > gpurun_out/${T}_pmc_k3.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_k3.log; exit 1; }
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > gpurun_out/${T}_cfg4.log 2> gpurun_out/${T}_cfg4.err || { tail -20 gpurun_out/${T}_cfg4.err; exit 1; }
grep '^{' gpurun_out/${T}_cfg4.log | tail -1 > gpurun_out/${T}_cfg4_bench_line.json; head -c 400 gpurun_out/${T}_cfg4_bench_line.json; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps > gpurun_out/prof_${T}.log 2>&1 || { tail -5 gpurun_out/prof_${T}.log; exit 1; }
echo "rocprof ok"
for c in cfg2 cfg3; do
  timeout -k 10 900 python bench.py --config $c --steps 30 --warmup 3 > gpurun_out/${T}_$c.log 2> gpurun_out/${T}_$c.err || { tail -20 gpurun_out/${T}_$c.err; exit 1; }
  grep '^{' gpurun_out/${T}_$c.log | tail -1 > gpurun_out/${T}_${c}_bench_line.json; head -c 300 gpurun_out/${T}_${c}_bench_line.json; echo
done
timeout -k 10 400 python bench.py --config cfg5 --steps 300 --warmup 20 > gpurun_out/${T}_cfg5.log 2>&1 || { tail -20 gpurun_out/${T}_cfg5.log; exit 1; }
grep '^{' gpurun_out/${T}_cfg5.log | tail -1 > gpurun_out/${T}_cfg5_bench_line.json; head -c 300 gpurun_out/${T}_cfg5_bench_line.json; echo
