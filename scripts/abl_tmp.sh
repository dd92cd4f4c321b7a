cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/evpmc_*
for c in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_BRANCH" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/evpmc_$tag -o k -- python3 scripts/eval_target.py > gpurun_out/evpmc_$tag.log 2>&1 || exit 1
  echo "$tag ok"
done
