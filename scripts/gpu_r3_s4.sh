#!/bin/bash
# A/B of the bf16x6 wgrad's prefetch depth (HGNN_X6_WG_PF = 1 | 2) at cfg4 shapes, K3 parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "linear or k3" > gpurun_out/t4.log 2>&1 || { tail -30 gpurun_out/t4.log; exit 1; }
tail -1 gpurun_out/t4.log
for v in 1 2 1 2; do
  HGNN_X6_WG_PF=$v timeout -k 10 120 python scripts/k3_ab.py --rows 9000000 --k 128 --bwd || exit 1
  HGNN_X6_WG_PF=$v timeout -k 10 120 python scripts/k3_ab.py --rows 1000000 --k 128 --bwd || exit 1
  HGNN_X6_WG_PF=$v timeout -k 10 120 python scripts/k3_ab.py --rows 9000000 --k 256 --segs 2 --bwd || exit 1
done
for v in 1 2; do
  HGNN_X6_WG_PF=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b4_$v.log 2>&1 || { tail -20 gpurun_out/b4_$v.log; exit 1; }
  echo "PF=$v"; grep '^{' gpurun_out/b4_$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items() if 'linear' in n})"
done
