cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --same-device --no-cpu-baseline > gpurun_out/bench_n2_rehearsal.log 2>&1; rc=$?; echo "n2 rehearsal rc=$rc"; tail -2 gpurun_out/bench_n2_rehearsal.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
