set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "loss or negativ or draw or score" > gpurun_out/t2.log 2>&1 || { tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
bash scripts/gpu_x6hb.sh > gpurun_out/x6hb.log 2>&1 || { tail -20 gpurun_out/x6hb.log; exit 1; }
cat gpurun_out/x6hb.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench2.log 2>&1 || { tail -20 gpurun_out/bench2.log; exit 1; }
grep '^{' gpurun_out/bench2.log | tail -1 | cut -c1-400
