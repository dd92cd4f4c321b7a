#!/bin/bash
# A/B of two in-tree library builds on the smaller configs (cfg2, cfg3): bench ms/step and the
# loss/gather kernels.  usage: LIBS="libhgnn_pre.so libhgnn.so" bash scripts/gpu_lib_ab_cfg.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in cfg2 cfg3; do
  for rep in 1 2; do
    for lib in $LIBS; do
      HGNN_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 \
        --no-cpu-baseline --json-out gpurun_out/abc_${cfg}_${rep}_${lib%.so}.json \
        > gpurun_out/abc.log 2>&1 || exit $?
      python - gpurun_out/abc_${cfg}_${rep}_${lib%.so}.json "$cfg $lib" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], d["ms_per_step"], {n: v["ms_per_step"] for n, v in d["kernels"].items()
                                      if n.startswith(("gather", "score", "edge"))})
PY
    done
  done
done
