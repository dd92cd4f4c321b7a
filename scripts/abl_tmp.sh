cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "loss or golden or shard or score or gather" > gpurun_out/t_sc.log 2>&1 || { tail -30 gpurun_out/t_sc.log; exit 1; }
tail -1 gpurun_out/t_sc.log
timeout -k 10 300 python scripts/microbench.py > gpurun_out/mb_sc.log 2>&1 || exit 1
grep "loss" gpurun_out/mb_sc.log | head -8
