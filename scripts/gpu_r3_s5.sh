#!/bin/bash
# A/B: XCD-aware tile order in the radix count kernel (libhgnn_base.so = without), sort tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_edges.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "sort or draw or csr or coo" > gpurun_out/t5.log 2>&1 || { tail -30 gpurun_out/t5.log; exit 1; }
tail -1 gpurun_out/t5.log
for lib in libhgnn_base.so libhgnn.so libhgnn_base.so libhgnn.so; do
  echo "== $lib"; HGNN_LIB=$lib timeout -k 10 120 python scripts/sort_bench.py --mode draw || exit 1
done
for lib in libhgnn_base.so libhgnn.so; do
  HGNN_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b5_$lib.log 2>&1 || { tail -20 gpurun_out/b5_$lib.log; exit 1; }
  echo "$lib"; grep '^{' gpurun_out/b5_$lib.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['ms_per_step'], k['sort_negatives']['ms_per_step'])"
done
