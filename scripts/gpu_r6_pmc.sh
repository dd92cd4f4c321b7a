#!/bin/bash
# Round-6 PMC passes (each counter its own rocprofv3 run, kernel-trace only): the cfg4 step's HBM
# bytes per kernel (FETCH_SIZE / WRITE_SIZE) merged with the four 9M-row K3 launches' bytes ->
# gpurun_out/pmc_r6.json (committed as profiles/pmc_r6.json; bench.py's `traffic`), and the K3
# cycle counters -> gpurun_out/pmc_k3_cfg4_r6.json (bench.py's projection `mfma_util`).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash scripts/pmc_r2.sh || exit 1
cp gpurun_out/pmc_step_cfg4.json gpurun_out/pmc_r6.json
bash scripts/pmc_k3_traffic.sh > gpurun_out/r6_pmc_k3_traffic.log 2>&1 || { tail -5 gpurun_out/r6_pmc_k3_traffic.log; exit 1; }
python3 scripts/pmc_k3_traffic_summarize.py gpurun_out/pmck3_fetch gpurun_out/pmck3_write gpurun_out/pmck3_fetch.log --merge gpurun_out/pmc_r6.json > /dev/null || exit 1
TAG=r6 bash scripts/pmc_k3_xs.sh > gpurun_out/r6_pmc_k3.log 2>&1 || { tail -5 gpurun_out/r6_pmc_k3.log; exit 1; }
rm -rf gpurun_out/pmcs_fetch gpurun_out/pmcs_write gpurun_out/pmck3_fetch gpurun_out/pmck3_write gpurun_out/pmcxs_r6_*
echo "pmc ok"
