cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; export TMPDIR=/tmp
for b in 6 7 8 9; do
  echo "bits=$b"
  HGNN_SORT_BITS=$b HGNN_SORT_LSD=1 timeout -k 10 60 python scripts/sort_bench.py || exit 1
  HGNN_SORT_BITS=$b timeout -k 10 60 python scripts/sort_bench.py || exit 1
done
for cfg in "6" "9"; do set -- $cfg
HGNN_SORT_BITS=$1 HGNN_SORT_LSD=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sortprof_$1 -o run -- python scripts/sort_bench.py --reps 5 > gpurun_out/sortprof.log 2>&1 || exit 1
python - gpurun_out/sortprof_$1/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'hgnn' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
done
