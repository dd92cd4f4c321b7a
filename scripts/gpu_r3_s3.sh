#!/bin/bash
# Round-3 session-2 A/B: new scoring entry test; rows in flight of the d = 128 gathers at cfg4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "draw" > gpurun_out/t3.log 2>&1 || { tail -30 gpurun_out/t3.log; exit 1; }
tail -1 gpurun_out/t3.log
i=0
for v in "HGNN_SC_U=4" "HGNN_SC_U=2" "HGNN_SC_U=3" "HGNN_SC_U=4" "HGNN_SC_U=2" "HGNN_SC_U=3"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$i.log 2>&1 || { tail -20 gpurun_out/b_$i.log; exit 1; }
  echo "$v"; grep '^{' gpurun_out/b_$i.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['ms_per_step'], {n[:24]: v['ms_per_step'] for n, v in k.items() if 'gather' in n or 'score' in n})"
done
