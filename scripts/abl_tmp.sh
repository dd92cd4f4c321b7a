cd $GRAFT_REPO_ROOT
for a in 0 1 2 4 7; do echo "ABL=$a"; HGNN_SCORE_ABL=$a timeout -k 10 300 python scripts/microbench.py --reps 10 2>&1 | grep "loss/"; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mb -o mb -- python scripts/microbench.py --reps 5 > gpurun_out/prof_mb.log 2>&1
echo rocprof $?
