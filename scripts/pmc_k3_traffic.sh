#!/bin/bash
# HBM bytes of the four 9M-row K3 launches (FETCH_SIZE, WRITE_SIZE: one --pmc pass each over
# scripts/k3_xs_target.py), summarised against the timer's algorithmic bytes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmck3_fetch -o f -- python3 scripts/k3_xs_target.py > gpurun_out/pmck3_fetch.log 2>&1 || { echo "fetch rc=$?"; tail -3 gpurun_out/pmck3_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmck3_write -o w -- python3 scripts/k3_xs_target.py > gpurun_out/pmck3_write.log 2>&1 || { echo "write rc=$?"; tail -3 gpurun_out/pmck3_write.log; exit 1; }
python3 scripts/pmc_k3_traffic_summarize.py gpurun_out/pmck3_fetch gpurun_out/pmck3_write gpurun_out/pmck3_fetch.log > gpurun_out/pmc_k3_traffic.json || exit 1
cat gpurun_out/pmc_k3_traffic.json
