#!/bin/bash
# Round-5 closing pass C: PMC HBM traffic of the cfg4 step (FETCH_SIZE / WRITE_SIZE passes ->
# profiles/pmc_r5.json, which bench.py reads for `traffic`), LDS bank conflicts per kernel, and
# the K3 counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash scripts/pmc_r2.sh || exit 1
bash scripts/pmc_lds_step.sh > gpurun_out/r5_lds_conflicts.txt || exit 1
cat gpurun_out/r5_lds_conflicts.txt | head -12
TAG=r5 bash scripts/pmc_k3_xs.sh > gpurun_out/r5_pmc_k3.log 2>&1 || { tail -5 gpurun_out/r5_pmc_k3.log; exit 1; }
echo "k3 pmc ok"
