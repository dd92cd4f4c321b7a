cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "linear or golden" > gpurun_out/t_f4.log 2>&1 || { tail -30 gpurun_out/t_f4.log; exit 1; }
tail -1 gpurun_out/t_f4.log
timeout -k 10 300 python scripts/microbench.py > gpurun_out/mb_f4.log 2>&1 || exit 1
grep "K3" gpurun_out/mb_f4.log | head -3
rm -rf gpurun_out/k3pmc_*
for c in "SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/k3pmc_$tag -o k -- python3 scripts/k3_target.py > gpurun_out/k3pmc_$tag.log 2>&1 || exit 1
  echo "$tag ok"
done
