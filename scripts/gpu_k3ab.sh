#!/bin/bash
# A/B of K3 kernel variants at cfg4 shapes: each line of VARIANTS is an env assignment list.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
while IFS= read -r v; do
  [ -z "$v" ] && continue
  echo "== $v"
  env $v timeout -k 10 200 python scripts/k3_bench.py --rows ${ROWS:-9000000} --shapes ${SHAPES:-128:128,256:128} --reps 10 || exit $?
done <<< "$VARIANTS"
