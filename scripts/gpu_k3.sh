cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
echo old; HGNN_LIB=libhgnn_old.so timeout -k 10 120 python scripts/k3_bench.py || exit 1
echo new; timeout -k 10 120 python scripts/k3_bench.py || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu -k "linear or golden" 2>&1 | tail -2
