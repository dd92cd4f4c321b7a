#!/bin/bash
# Round 5: the K = 384 / 512 split path (cfg5): K3 parity tests, the mini-batch / cfg5 GPU tests,
# and the cfg5 bench line with its per-kernel rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
# (-k applies to every file named, so the K3 selection and the mini-batch files run separately)
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "linear or k3" -m gpu > gpurun_out/wide_tests.log 2>&1 || { tail -30 gpurun_out/wide_tests.log; exit 1; }
tail -1 gpurun_out/wide_tests.log
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_minibatch_graph.py tests/test_full_size_cfg5.py tests/test_sampler.py -m gpu > gpurun_out/wide_mb_tests.log 2>&1 || { tail -30 gpurun_out/wide_mb_tests.log; exit 1; }
tail -1 gpurun_out/wide_mb_tests.log
timeout -k 10 300 python bench.py --config cfg5 --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/wide_cfg5.log 2>&1 || { tail -5 gpurun_out/wide_cfg5.log; exit 1; }
grep '^{' gpurun_out/wide_cfg5.log | tail -1 > gpurun_out/wide_cfg5_line.json
python3 -c "
import json; d=json.load(open('gpurun_out/wide_cfg5_line.json')); print('cfg5', d['ms_per_step'], d['value'])
for k,v in sorted(d.get('kernels',{}).items()): print(k, v['ms_per_step'], v['launches'])"
