#!/bin/bash
# A/B: the x6 forward with its five small products in two interleaved accumulators
# (HGNN_X6_SPLITLO = 1) at K = 256; K3 parity tests under it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
HGNN_X6_SPLITLO=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "linear or k3 or golden or step" > gpurun_out/t8.log 2>&1 || { tail -30 gpurun_out/t8.log; exit 1; }
tail -1 gpurun_out/t8.log
for rep in 1 2; do
  for v in 0 1; do
    echo "== SPLITLO=$v"
    HGNN_X6_SPLITLO=$v timeout -k 10 120 python scripts/k3_ab.py --rows 9000000 --k 256 --segs 2 || exit 1
    HGNN_X6_SPLITLO=$v timeout -k 10 120 python scripts/k3_ab.py --rows 1000000 --k 256 --segs 2 || exit 1
  done
done
for v in 0 1; do
  HGNN_X6_SPLITLO=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b8_$v.log 2>&1 || { tail -20 gpurun_out/b8_$v.log; exit 1; }
  echo "SPLITLO=$v"; grep '^{' gpurun_out/b8_$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'linear_fwd' in n})"
done
