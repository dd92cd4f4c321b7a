#!/bin/bash
# Per-kernel HBM traffic of the cfg4 training step (FETCH_SIZE, WRITE_SIZE passes) and the K3
# MFMA busy fraction at d=h=128 (k3_target.py cfg4 shapes).  Each pass its own run, kernel-trace only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
CFG=${CFG:-cfg4}
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcs_fetch -o f -- python3 scripts/pmc_step_target.py $CFG 2 > gpurun_out/pmcs_fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcs_write -o w -- python3 scripts/pmc_step_target.py $CFG 2 > gpurun_out/pmcs_write.log 2>&1 || exit $?
python3 scripts/pmc_step_summarize.py gpurun_out/pmcs_fetch gpurun_out/pmcs_write gpurun_out/pmcs_fetch.log gpurun_out/pmc_step_$CFG.json > /dev/null || exit $?
echo "summary written"
