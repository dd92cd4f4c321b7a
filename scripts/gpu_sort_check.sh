cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu -k "sort or csr or loss or sampler" > gpurun_out/sort_tests.log 2>&1; rc=$?; tail -4 gpurun_out/sort_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/sort_bench.py && HGNN_SORT_LSD=1 timeout -k 10 120 python scripts/sort_bench.py && timeout -k 10 120 python scripts/sort_bench.py --keys 800000
