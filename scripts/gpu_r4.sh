#!/bin/bash
# Round-4 measurement pass (one GPU call): the cfg4 bench line, the K3 per-launch bench at the
# cfg4 shapes, a rocprofv3 kernel-stats profile of the bench and the K3 PMC passes.  Each GPU step
# under its own time limit; stops at the first failure.
#   STEPS="bench k3 prof pmc" (default: all four) selects the steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r4}
S=" ${STEPS:-bench k3 prof pmc} "
if [[ $S == *" bench "* ]]; then
  timeout -k 10 900 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/${TAG}_cfg4.log 2> gpurun_out/${TAG}_cfg4.err || { tail -20 gpurun_out/${TAG}_cfg4.err; exit 1; }
  grep '^{' gpurun_out/${TAG}_cfg4.log | tail -1 > gpurun_out/${TAG}_cfg4_bench_line.json
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_cfg4_bench_line.json'));print(d['ms_per_step'],d['value'],d['roofline']['frac'],d.get('cpu_baseline'));[print(k,v['ms_per_step']) for k,v in d['kernels'].items() if k.startswith(('linear','sort','edge','score'))]"
fi
if [[ $S == *" k3 "* ]]; then
  timeout -k 10 300 python -u scripts/k3_xs_bench.py > gpurun_out/${TAG}_k3_xs.jsonl 2>&1 || { tail -20 gpurun_out/${TAG}_k3_xs.jsonl; exit 1; }
  cat gpurun_out/${TAG}_k3_xs.jsonl
fi
if [[ $S == *" prof "* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run \
    -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps > gpurun_out/prof_${TAG}.log 2>&1 || { tail -5 gpurun_out/prof_${TAG}.log; exit 1; }
  echo "rocprof ok"
fi
if [[ $S == *" pmc "* ]]; then
  TAG=$TAG bash scripts/pmc_k3_xs.sh > gpurun_out/${TAG}_pmc_k3.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_k3.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/pmc_k3_cfg4_${TAG}.json'));[print(k,v.get('mfma_util'),v.get('valu_per_mfma')) for k,v in d['kernels'].items()]"
fi
