cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "linear or golden" > gpurun_out/t_v4.log 2>&1 || { tail -30 gpurun_out/t_v4.log; exit 1; }
tail -1 gpurun_out/t_v4.log
timeout -k 10 300 python scripts/microbench.py > gpurun_out/mb_v4.log 2>&1 || exit 1
grep K3 gpurun_out/mb_v4.log
HGNN_LIN_V3=1 timeout -k 10 300 python scripts/microbench.py > gpurun_out/mb_v3.log 2>&1 || exit 1
grep "K3 bwd" gpurun_out/mb_v3.log
