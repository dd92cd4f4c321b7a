#!/bin/bash
# Round-3 closing pass on the final build (one GPU call): the whole -m gpu suite + smoke, PMC
# traffic of the cfg4 step (-> profiles/pmc_r3.json), the cfg4 bench line with its CPU baseline, a rocprofv3 kernel-stats profile of the same bench, cfg2 / cfg3
# / cfg5 lines.  Each GPU step under its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/gpu_tests.log; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash scripts/pmc_r2.sh || exit $?
cp gpurun_out/pmc_step_cfg4.json profiles/pmc_r3.json && cp gpurun_out/pmc_step_cfg4.json gpurun_out/pmc_r3.json
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > gpurun_out/f_cfg4.log 2> gpurun_out/f_cfg4.err || { tail -20 gpurun_out/f_cfg4.err; exit 1; }
grep '^{' gpurun_out/f_cfg4.log | tail -1 > gpurun_out/f_cfg4_bench_line.json; head -c 400 gpurun_out/f_cfg4_bench_line.json; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps > gpurun_out/prof_f.log 2>&1 || { tail -5 gpurun_out/prof_f.log; exit 1; }
echo "rocprof ok"
for c in cfg2 cfg3; do
  timeout -k 10 900 python bench.py --config $c --steps 30 --warmup 3 > gpurun_out/f_$c.log 2> gpurun_out/f_$c.err || { tail -20 gpurun_out/f_$c.err; exit 1; }
  grep '^{' gpurun_out/f_$c.log | tail -1 > gpurun_out/f_${c}_bench_line.json; head -c 300 gpurun_out/f_${c}_bench_line.json; echo
done
timeout -k 10 300 python bench.py --config cfg5 --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/f_cfg5.log 2>&1 || { tail -20 gpurun_out/f_cfg5.log; exit 1; }
grep '^{' gpurun_out/f_cfg5.log | tail -1 > gpurun_out/f_cfg5_bench_line.json; head -c 300 gpurun_out/f_cfg5_bench_line.json; echo
