#!/bin/bash
# PMC traffic of the roofline kernel: two --pmc passes (kernel-trace only), then summarise.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python3 scripts/pmc_target.py > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python3 scripts/pmc_target.py > gpurun_out/pmc_write.log 2>&1 || exit $?
python3 scripts/pmc_summarize.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_fetch.log > gpurun_out/pmc_gather.json && cat gpurun_out/pmc_gather.json
