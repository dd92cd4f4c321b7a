cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider -k "linear or golden" > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -le 1 ] || exit $rc
for v in 0 1; do echo "HGNN_LIN_GENERAL=$v"; HGNN_LIN_GENERAL=$v timeout -k 10 300 python scripts/microbench.py --reps 10 2>&1 | grep "K3"; done
