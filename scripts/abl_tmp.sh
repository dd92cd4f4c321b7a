cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "loss or golden or shard or score or sort or csr" > gpurun_out/t_so.log 2>&1 || { tail -30 gpurun_out/t_so.log; exit 1; }
tail -1 gpurun_out/t_so.log
timeout -k 10 300 python scripts/microbench.py > gpurun_out/mb_so.log 2>&1 || exit 1
grep "loss" gpurun_out/mb_so.log | head -6
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_so.log 2>&1 || exit 1
tail -1 gpurun_out/b_so.log | cut -c1-200
