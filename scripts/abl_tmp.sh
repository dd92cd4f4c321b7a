cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "linear or golden" > gpurun_out/t_lin.log 2>&1 || { tail -30 gpurun_out/t_lin.log; exit 1; }
tail -1 gpurun_out/t_lin.log
timeout -k 10 300 python scripts/microbench.py --config cfg3 > gpurun_out/mb_c3.log 2>&1 || exit 1
grep "K3" gpurun_out/mb_c3.log | head -5
