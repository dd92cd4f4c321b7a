#!/bin/bash
# Where the split-once K3 kernels' cycles go at the cfg4 9M-row shapes (scripts/k3_xs_target.py):
# MFMA busy, wave-cycle breakdown, instruction mix, LDS conflicts.  Separate --pmc passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4}
i=0
for c in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
         "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
         "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmcxs_${TAG}_$i -o k -- python3 scripts/k3_xs_target.py > gpurun_out/pmcxs_${TAG}_$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 gpurun_out/pmcxs_${TAG}_$i.log; exit 1; }
done
export TAG
python3 scripts/pmc_xs_summarize.py $TAG > gpurun_out/pmc_k3_cfg4_${TAG}.json && cat gpurun_out/pmc_k3_cfg4_${TAG}.json
