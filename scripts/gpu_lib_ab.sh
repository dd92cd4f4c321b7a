#!/bin/bash
# A/B of two in-tree builds of the library on the cfg4 step (bench.py, HIP-event per-kernel
# timer run included): usage LIBS="libhgnn.so libhgnn_nt.so" bash scripts/gpu_lib_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
i=0
for rep in 1 2; do
  for lib in $LIBS; do
    i=$((i+1))
    HGNN_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
      --json-out gpurun_out/ab_${i}_${lib%.so}.json > gpurun_out/ab_${i}.log 2>&1 || exit $?
    python - gpurun_out/ab_${i}_${lib%.so}.json "$lib" <<'PY'
import json, os, sys
d = json.load(open(sys.argv[1]))
k = d["kernels"]
print(sys.argv[2], d["ms_per_step"], {n: v["ms_per_step"] for n, v in k.items()
                                      if n.startswith(tuple(os.environ.get("AB_KERNELS", "gather,score,edge").split(",")))})
PY
  done
done
