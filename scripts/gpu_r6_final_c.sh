#!/bin/bash
# Round-6 closing pass C: PMC HBM traffic of the cfg4 step (FETCH_SIZE / WRITE_SIZE passes ->
# gpurun_out/pmc_step_cfg4.json, merged into profiles/pmc_r6.json, which bench.py reads for
# `traffic`) and the K3 counters (-> profiles/pmc_k3_cfg4_r6.json, read for `mfma_util`).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
[ -n "$NO_STEP" ] || bash scripts/pmc_r2.sh || exit 1
TAG=${TAG:-r6} bash scripts/pmc_k3_xs.sh > gpurun_out/${TAG:-r6}_pmc_k3.log 2>&1 || { tail -5 gpurun_out/${TAG:-r6}_pmc_k3.log; exit 1; }
echo "k3 pmc ok"
